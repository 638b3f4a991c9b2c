#!/bin/bash
# GPU checkpoint: the -m gpu suite, then the BASELINE configs[3] bench line (log-MAP).
set -o pipefail
O=gpurun_out/${TAG:-r03a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --mod 8PSK --rate 1/2 --algo log-map --batch 1048576 --steps 3 --warmup 1 > $O/c3_8psk_logmap.json 2> $O/c3.err
rc=$?
cat $O/c3_8psk_logmap.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['decode_kernel_ms'], d['roofline']['frac'])"
exit $rc
