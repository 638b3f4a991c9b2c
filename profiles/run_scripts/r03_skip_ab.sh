#!/bin/bash
# A/B: decoder 1 skips the dead extrinsic at rows outside perm's image (TDEC_SKIP_UNUSED)
#   libtdec_base.so = HEAD before the change (tools/build_rev.sh), libtdec.so = working tree
set -o pipefail
O=gpurun_out/${TAG:-r03sk}; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 300 python tools/ab.py $L/libtdec_base.so $L/libtdec.so --batch 1048576 --rounds 3 > $O/ab_ml.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml.log
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_base.so --batch 1048576 --rounds 3 > $O/ab_ml_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_ml_r.log
timeout -k 10 200 python tools/ab.py $L/libtdec_base.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 5 > $O/ab_c1.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_c1.log
timeout -k 10 300 python tools/ab.py $L/libtdec_base.so $L/libtdec.so --algo 1 --mod 8PSK --rate 1/2 --batch 262144 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
