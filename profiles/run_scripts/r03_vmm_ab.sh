#!/bin/bash
# Workspace placement: default (shuffled 64 MiB VMM chunks) vs one hipMalloc vs the probe, fresh processes
set -o pipefail
O=gpurun_out/${TAG:-r03n}
mkdir -p $O
for i in 1 2 3; do
  for cfg in "TDEC_WS_ALLOC=vmm" "TDEC_WS_ALLOC=malloc" "TDEC_PLACEMENT_PROBE=1"; do
    env $cfg timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > $O/run.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/run.json')); print('$cfg run $i', round(d['value']), round(d['decode_kernel_ms'], 2))" | tee -a $O/vmm_ab.txt
  done
done
