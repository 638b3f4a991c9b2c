#!/bin/bash
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
L=modulations_amd/lib
TDEC_WAVE_DUMP=$O/c1.txt timeout -k 10 200 python tools/wave_dump.py $L/libtdec_wt4.so $L/libtdec_wt1.so --batch 102400 > $O/c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/c1.log
TDEC_WAVE_DUMP=$O/c1b.txt timeout -k 10 200 python tools/wave_dump.py $L/libtdec_wt4.so --batch 51200 > $O/c1b.log 2>&1 || exit $?
grep -v amdgpu.ids $O/c1b.log
