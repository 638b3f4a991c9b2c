# Headline decoder knobs re-measured on this round's kernel (in-process A/B, 262 144
# codewords, both orders): non-temporal workspace stores (nt), F1 rolling prefetch of
# 8 steps (roll8), F1 groups of 8 (fg8).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python -u tools/ab.py $L/libtdec.so $L/libtdec_nt.so $L/libtdec_roll8.so $L/libtdec_fg8.so --rounds 6 > $O/ab_a.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab.py $L/libtdec_fg8.so $L/libtdec_roll8.so $L/libtdec_nt.so $L/libtdec.so --rounds 6 > $O/ab_b.txt 2>&1 || exit 1
