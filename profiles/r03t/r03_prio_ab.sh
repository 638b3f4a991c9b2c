#!/bin/bash
# A/B: issue priority by tile progress (TDEC_PRIO=1) against the default build.
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_prio.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 200 python tools/ab.py $L/libtdec_prio.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1r.log
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_prio.so --n 212 --mod QPSK --batch 131072 --rounds 3 > $O/ab_c1b.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1b.log
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_prio.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_prio.so --rate 1/2 --mod 8PSK --algo 1 --batch 262144 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
