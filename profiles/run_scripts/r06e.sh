# Round 6: the opaque workspace row stride (v_add_lshl_u32 addressing as in round 5)
# against round 5's library, configs[2] at the bench's 1 M codewords and configs[1],
# both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 600 python tools/ab.py $L/libtdec_r05.so $L/libtdec.so --batch 1048576 --rounds 4 > $O/ab_c2.txt 2>&1 || exit 1
timeout -k 10 600 python tools/ab.py $L/libtdec.so $L/libtdec_r05.so --batch 1048576 --rounds 4 > $O/ab_c2_rev.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_r05.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 8 > $O/ab_c1.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_r05.so --n 212 --mod QPSK --batch 102400 --rounds 8 > $O/ab_c1_rev.txt 2>&1 || exit 1
echo r06e done
