# Round 5: what the log-MAP definition's bounded-grid max* (the +8 that lets the
# oracle pin v_exp_f32 / v_log_f32 exactly) costs: the same decoder with max* =
# max + log2(1 + 2^-|a-b|) (TDEC_LM_FAST, different bits), both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_lmfast.so --batch 262144 --rate 1/2 --algo 1 --mod 8PSK --rounds 4 > $O/ab_a.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_lmfast.so $L/libtdec.so --batch 262144 --rate 1/2 --algo 1 --mod 8PSK --rounds 4 > $O/ab_b.log 2>&1 || exit 1
