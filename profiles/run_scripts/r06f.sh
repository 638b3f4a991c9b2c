# Round 6: log-MAP recursions with the predecessor / successor sums two per
# v_pk_add_f32 (TDEC_LM_PAIR: same operations, same bits) against the shipped
# library at configs[3], in one process, both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
L=modulations_amd/lib
A="--n 752 --rate 1/2 --mod 8PSK --algo 1"
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_lmpair2.so $A --rounds 4 > $O/ab_c3.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_lmpair2.so $L/libtdec.so $A --rounds 4 > $O/ab_c3_rev.txt 2>&1 || exit 1
echo r06f done
