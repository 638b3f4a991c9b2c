#!/bin/bash
# A/B: policy-4 priority with 4 progress units per SISO (TDEC_PRIO_FINE=1) vs 2 (default)
set -o pipefail
O=gpurun_out/r03ab; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_fine.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 200 python tools/ab.py $L/libtdec_fine.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1r.log
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_fine.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
