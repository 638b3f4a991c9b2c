#!/bin/bash
# A/B: B1 skips its top windows' extrinsics (TDEC_B1_TOP): libtdec_sk.so = HEAD without it,
# libtdec.so = margin 2 windows, libtdec_top4.so = margin 4; then the GPU suite on libtdec.so.
set -o pipefail
O=gpurun_out/${TAG:-r03top}; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python tools/ab.py $L/libtdec_sk.so $L/libtdec.so $L/libtdec_top4.so --batch 1048576 --rounds 4 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 400 python tools/ab.py $L/libtdec_top4.so $L/libtdec.so $L/libtdec_sk.so --batch 1048576 --rounds 4 > $O/ab_ml_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml_r.log
timeout -k 10 200 python tools/ab.py $L/libtdec_sk.so $L/libtdec.so $L/libtdec_top4.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
