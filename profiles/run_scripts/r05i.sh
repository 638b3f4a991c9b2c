# Round 5: log-MAP decoder at three waves per SIMD (TDEC_LM_WPE=3; its inner loops now
# spill nothing) against two, both orders, configs[3] inputs (8PSK r=1/2 N=752).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_lm3.so --batch 262144 --rate 1/2 --algo 1 --mod 8PSK --rounds 4 > $O/ab_a.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_lm3.so $L/libtdec.so --batch 262144 --rate 1/2 --algo 1 --mod 8PSK --rounds 4 > $O/ab_b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o calls --output-format csv -- python tools/call_probe.py > $O/probe.log 2>&1 || exit 1
