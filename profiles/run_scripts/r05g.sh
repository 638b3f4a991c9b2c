# Round 5: checkpoints every 16 steps (TDEC_CK16) re-measured after the spill removal.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_ck16.so --batch 1048576 --rounds 5 > $O/ab_c2_a.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_ck16.so $L/libtdec.so --batch 1048576 --rounds 5 > $O/ab_c2_b.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_ck16.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_a.log 2>&1 || exit 1
