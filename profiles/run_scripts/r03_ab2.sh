#!/bin/bash
# demap A/B (16 / 64 / 256QAM, gray arithmetic search vs scan) + demap GPU tests + max-log variants A/B
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -k "demap or fused" -x -q --timeout 120 --timeout-method thread > $O/demap_tests.log 2>&1; rc=$?
tail -3 $O/demap_tests.log
[ $rc -eq 0 ] || exit $rc
for m in 16QAM 64QAM 256QAM; do
  timeout -k 10 200 python tools/ab_demap.py modulations_amd/lib/libtdec.so modulations_amd/lib/libtdec_dmscan.so --mod $m --rounds 3 > $O/ab_dm_$m.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/ab_dm_$m.log
done
timeout -k 10 600 python tools/ab.py modulations_amd/lib/libtdec.so modulations_amd/lib/libtdec_nt.so modulations_amd/lib/libtdec_w4.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1
grep -v amdgpu.ids $O/ab_ml.log
