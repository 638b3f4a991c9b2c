#!/bin/bash
# GPU checkpoint: the -m gpu suite, then the headline bench (+ probe A/B when PROBE=1)
set -o pipefail
O=gpurun_out/${TAG:-r03}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python - <<PY
import json; d=json.load(open("$O/bench.json"))
print("value", d["value"], "decode ms", d["decode_kernel_ms"], "frac", d["roofline"]["frac"])
print(json.dumps(d.get("host_api"), indent=1)); print("cpu", d["cpu_baseline"]["value"], "spot", d["parity_spot_check"])
PY
