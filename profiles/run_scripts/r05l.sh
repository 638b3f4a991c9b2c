# Round 5: the item queue with the pusher yielding to waiting waves (TDEC_IQ_YIELD ~4 / 16 us;
# iqy0 = no yield) against whole tiles per wave (libtdec.so) and the previous revision.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
L=modulations_amd/lib
TDEC_ITEMQ=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_properties.py > $O/tests_iq.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_iq.so $L/libtdec_iqy16.so $L/libtdec_iqy0.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_a.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_iqy16.so $L/libtdec_iq.so $L/libtdec.so $L/libtdec_iqy0.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_b.log 2>&1 || exit 1
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_iq.so $L/libtdec_iqy16.so $L/libtdec_prev.so --batch 1048576 --rounds 4 > $O/ab_c2_a.log 2>&1 || exit 1
