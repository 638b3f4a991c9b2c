#!/bin/bash
# A/B: rolling F1 prefetch (TDEC_F1_ROLL=16 / 8) vs grouped (default)
set -o pipefail
O=gpurun_out/r03ae; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_r16.so $L/libtdec_r8.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_r16.so $L/libtdec_r8.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
