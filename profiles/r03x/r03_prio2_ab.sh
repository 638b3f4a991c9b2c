#!/bin/bash
# A/B of the issue-priority policies (TDEC_PRIO 1 default / 2 by pass / 3 both / 0 none)
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_p2.so $L/libtdec_p3.so $L/libtdec_p0.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_p2.so $L/libtdec_p3.so $L/libtdec_p0.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
