#!/bin/bash
set -o pipefail
O=gpurun_out/r03ah; mkdir -p $O
L=modulations_amd/lib
for m in 16QAM 256QAM; do
  timeout -k 10 200 python tools/ab_demap.py $L/libtdec_old.so $L/libtdec_dmall.so $L/libtdec_dm32.so $L/libtdec.so --mod $m --rounds 3 > $O/ab_$m.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab_$m.log
done
