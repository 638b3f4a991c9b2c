#!/bin/bash
# Fresh-process bench pairs, base (HEAD before the dead-extrinsic skip) vs the current library.
set -o pipefail
O=gpurun_out/${TAG:-r03sk4}; mkdir -p $O
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export TDEC_LIB_VARIANT=base; else unset TDEC_LIB_VARIANT; fi
    timeout -k 10 200 python -u bench.py --no-cpu --steps 5 --warmup 1 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit $?
    python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v run $i', round(d['value']), round(d['decode_kernel_ms'], 2), round(d['ms_per_step'], 2))" | tee -a $O/bench_ab.txt
  done
done
rocm-smi --showclocks --showpower --showtemp > $O/smi.txt 2>&1 || true
