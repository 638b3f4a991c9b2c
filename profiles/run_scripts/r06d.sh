# Round 6: configs[3] libraries in one process (round 4's final
# library, round 5's, round 6's -- settles 2.21 -> 2.05 M), and a timing-only
# variant whose log-MAP extrinsic takes one 16-term log-sum per input class instead
# of two levels of lse4 (x16: different bits).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
L=modulations_amd/lib
A="--n 752 --rate 1/2 --mod 8PSK --algo 1"
timeout -k 10 500 python tools/ab.py $L/libtdec_r04.so $L/libtdec_r05.so $L/libtdec.so $A --rounds 4 > $O/ab_c3_r04_r05_r06.txt 2>&1 || exit 1
timeout -k 10 500 python tools/ab.py $L/libtdec.so $L/libtdec_r05.so $L/libtdec_r04.so $A --rounds 4 > $O/ab_c3_r06_r05_r04.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_x16.so $A --rounds 4 > $O/ab_c3_x16.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_x16.so $L/libtdec.so $A --rounds 4 > $O/ab_c3_x16_rev.txt 2>&1 || exit 1
timeout -k 10 500 python tools/ab.py $L/libtdec_r04.so $L/libtdec_r05.so $L/libtdec.so --rounds 4 > $O/ab_c2_r04_r05_r06.txt 2>&1 || exit 1
echo r06d done
