#!/bin/bash
# A/B #2 of TDEC_SKIP_UNUSED: fresh bench processes alternating base / new, longer
# in-process A/B in both orders, and the midpoint-skip variant (TDEC_SKIP_MID=1).
set -o pipefail
O=gpurun_out/${TAG:-r03sk2}; mkdir -p $O
L=modulations_amd/lib
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export TDEC_LIB_VARIANT=base; else unset TDEC_LIB_VARIANT; fi
    timeout -k 10 200 python -u bench.py --no-cpu --steps 5 --warmup 1 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit $?
    python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v run $i', round(d['value']), round(d['decode_kernel_ms'], 2), round(d['ms_per_step'], 2))" | tee -a $O/bench_ab.txt
  done
done
unset TDEC_LIB_VARIANT
timeout -k 10 400 python tools/ab.py $L/libtdec_base.so $L/libtdec.so $L/libtdec_mid2.so --batch 1048576 --rounds 5 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 400 python tools/ab.py $L/libtdec_mid2.so $L/libtdec.so $L/libtdec_base.so --batch 1048576 --rounds 5 > $O/ab_ml_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml_r.log
