# Round 5: A/B of the headline decoder's spill removal (saddr LDS DMAs + laundered lane in
# the backward prologues) against the round-4 code (old) and saddr alone, both orders,
# configs[2] (1 M codewords) and configs[1] (N = 212 QPSK, 102 400 codewords).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_old.so $L/libtdec_saddr.so --batch 1048576 --rounds 5 > $O/ab_c2_a.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_old.so $L/libtdec.so --batch 1048576 --rounds 5 > $O/ab_c2_b.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_old.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_a.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_old.so $L/libtdec.so --batch 102400 --n 212 --mod QPSK --rounds 8 > $O/ab_c1_b.log 2>&1 || exit 1
