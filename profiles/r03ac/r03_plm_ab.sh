#!/bin/bash
# A/B: policy-4 issue priority in the log-MAP decoder (TDEC_PRIO_LM=1) vs none (default)
set -o pipefail
O=gpurun_out/r03ac; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_plm.so --rate 1/2 --mod 8PSK --algo 1 --batch 1048576 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
timeout -k 10 500 python tools/ab.py $L/libtdec_plm.so $L/libtdec.so --rate 1/2 --mod 8PSK --algo 1 --batch 1048576 --rounds 3 > $O/ab_lm_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm_r.log
