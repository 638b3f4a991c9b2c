#!/bin/bash
# VMM workspace chunk size (TDEC_VMM_CHUNK_MB) in fresh bench processes, headline config
set -o pipefail
O=gpurun_out/r03af; mkdir -p $O
for rep in 1 2; do
  for mb in 64 16 32 128 512; do
    TDEC_VMM_CHUNK_MB=$mb timeout -k 10 200 python -u bench.py --no-cpu --steps 5 > $O/c${mb}_$rep.json 2> $O/c${mb}_$rep.err || exit $?
    python -c "import json;d=json.load(open('$O/c${mb}_$rep.json'));print('chunk $mb MB rep $rep', round(d['decode_kernel_ms'],2), round(d['value']/1e6,3))" | tee -a $O/chunk_ab.txt
  done
done
