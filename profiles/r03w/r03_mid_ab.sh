#!/bin/bash
set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_mid.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 400 python tools/ab.py $L/libtdec_mid.so $L/libtdec.so --batch 1048576 --rounds 3 > $O/ab_ml_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml_r.log
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_mid.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
