#!/bin/bash
set -o pipefail
O=gpurun_out/r03aj; mkdir -p $O
L=modulations_amd/lib
for m in 16QAM 256QAM QPSK; do
  timeout -k 10 200 python tools/ab_demap.py $L/libtdec.so $L/libtdec_dmpf.so --mod $m --rounds 3 > $O/ab_$m.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab_$m.log
done
