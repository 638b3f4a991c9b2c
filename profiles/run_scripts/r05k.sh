# Round 5: the (tile, iteration) item queue (TDEC_ITEMQ).  First its correctness on the
# throughput paths (GPU parity / full-size property tests with TDEC_ITEMQ=1), then
# in-process A/Bs: the flattened tile loop (libtdec.so) vs the previous revision
# (prev) vs the item queue (iq), configs[2] (1 M) and configs[1] (N = 212, 102 400).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
L=modulations_amd/lib
TDEC_ITEMQ=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_properties.py tests/test_gpu_parity.py tests/test_gpu_logmap.py > $O/tests_iq.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_prev.so $L/libtdec_iq.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_a.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_iq.so $L/libtdec_prev.so $L/libtdec.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_b.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_prev.so $L/libtdec_iq.so --batch 1048576 --rounds 4 > $O/ab_c2_a.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_iq.so $L/libtdec_prev.so $L/libtdec.so --batch 1048576 --rounds 4 > $O/ab_c2_b.log 2>&1 || exit 1
