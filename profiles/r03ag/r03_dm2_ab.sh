#!/bin/bash
# persistent k_demap_planes with symbol prefetch (working tree) vs HEAD: planes identical, time per launch
set -o pipefail
O=gpurun_out/r03ag; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -k "demap or fused or planes" -x -q --timeout 120 --timeout-method thread > $O/demap_tests.log 2>&1 || { tail -20 $O/demap_tests.log; exit 1; }
tail -1 $O/demap_tests.log
for m in 16QAM 256QAM QPSK 8PSK 64QAM; do
  timeout -k 10 200 python tools/ab_demap.py $L/libtdec.so $L/libtdec_old.so --mod $m --rounds 3 > $O/ab_$m.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab_$m.log
done
