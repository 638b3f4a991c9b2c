#!/bin/bash
# Round-3 evidence, part $1:
#   a: GPU suite + smoke + headline bench (host API, CPU baseline) + headline and configs[3] rocprof
#   b: configs[4] sweeps (both interleavers, JSON echoed) + placement-probe A/B in fresh processes
set -o pipefail
T=${TAG:-r03z}
O=gpurun_out/$T
mkdir -p $O
case $1 in
a)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
  timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['decode_kernel_ms'], d['roofline']['frac'], d['parity_spot_check']); print(json.dumps(d['host_api']))"
  TAG=$T ./tools/configs_r03.sh c2 c3 || exit 1
  ;;
b)
  TAG=$T ./tools/configs_r03.sh sweep || exit 1
  for f in $O\_sweep/*.json; do echo "== $f"; cat $f; done
  for i in 1 2 3; do
    for p in 0 1; do
      TDEC_PLACEMENT_PROBE=$p timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > $O/probe${p}_$i.json 2>> $O/probe.err || exit 1
      python -c "import json; d=json.load(open('$O/probe${p}_$i.json')); print('probe=$p run $i', round(d['value']), round(d['decode_kernel_ms'], 2))" | tee -a $O/probe_ab.txt
    done
  done
  ;;
esac
