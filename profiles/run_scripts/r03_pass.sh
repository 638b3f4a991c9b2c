#!/bin/bash
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 200 python tools/ab.py $L/libtdec_pt.so --batch 262144 --rounds 1 > $O/pt_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $O/pt_c2.log
timeout -k 10 200 python tools/ab.py $L/libtdec_pt.so --n 212 --mod QPSK --batch 102400 --rounds 1 > $O/pt_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/pt_c1.log
