#!/bin/bash
# A/B: issue priority against the SIMD's other wave (TDEC_PRIO=4) vs progress quarters (default)
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_p4.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 200 python tools/ab.py $L/libtdec_p4.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1r.log
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_p4.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
