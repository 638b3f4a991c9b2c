#!/bin/bash
# A/B: packed max* pairs in log-MAP (TDEC_LM_PK=1, default build) vs scalar (lmpk0)
set -o pipefail
O=gpurun_out/r03ad; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_logmap.py -x -q --timeout 120 --timeout-method thread > $O/lm_tests.log 2>&1 || { tail -20 $O/lm_tests.log; exit 1; }
tail -1 $O/lm_tests.log
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_lmpk0.so --rate 1/2 --mod 8PSK --algo 1 --batch 262144 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
timeout -k 10 400 python tools/ab.py $L/libtdec_lmpk0.so $L/libtdec.so --rate 1/2 --mod 8PSK --algo 1 --batch 262144 --rounds 3 > $O/ab_lm_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm_r.log
