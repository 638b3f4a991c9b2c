#!/bin/bash
# A/B of the tile decoders' block size (TDEC_DEC_WAVES 4 / 1 / 2): configs[1]
# (one round of tiles), the headline batch and log-MAP; same bits checked.
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_dw1.so $L/libtdec_dw2.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 200 python tools/ab.py $L/libtdec_dw1.so $L/libtdec.so $L/libtdec_dw2.so --n 212 --mod QPSK --batch 131072 --rounds 3 > $O/ab_c1b.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1b.log
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_dw1.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_dw1.so --rate 1/2 --mod 8PSK --algo 1 --batch 262144 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
