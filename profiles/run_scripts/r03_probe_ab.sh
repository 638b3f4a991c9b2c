#!/bin/bash
# Headline bench (host API, CPU baseline) + placement probe A/B in fresh processes.
set -o pipefail
O=gpurun_out/${TAG:-r03e}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
for i in 1 2 3; do
  for p in 0 1; do
    TDEC_PLACEMENT_PROBE=$p timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > $O/probe${p}_$i.json 2>> $O/probe.err || exit $?
    python -c "import json; d=json.load(open('$O/probe${p}_$i.json')); print('probe=$p run $i', round(d['value']), round(d['decode_kernel_ms'],2))" | tee -a $O/probe_ab.txt
  done
done
