#!/bin/bash
# demap of batch i+1 beside the decode of batch i (bench --overlap), configs[1] and the headline
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
for ov in no-overlap overlap no-overlap overlap; do
  timeout -k 10 120 python -u bench.py --mod QPSK --n 212 --batch 102400 --steps 20 --no-cpu --$ov > $O/c1_$ov.json 2> $O/c1_$ov.err || exit $?
  python -c "import json;d=json.load(open('$O/c1_$ov.json'));print('c1 $ov', round(d['ms_per_step'],3), round(d['decode_kernel_ms'],3), round(d['value']/1e6,3))"
done
for ov in no-overlap overlap; do
  timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --$ov > $O/c2_$ov.json 2> $O/c2_$ov.err || exit $?
  python -c "import json;d=json.load(open('$O/c2_$ov.json'));print('c2 $ov', round(d['ms_per_step'],3), round(d['decode_kernel_ms'],3), round(d['value']/1e6,3))"
done
