set -o pipefail
mkdir -p gpurun_out/r04r
export TMPDIR=/tmp
O=gpurun_out/r04r
L=modulations_amd/lib
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_lmw4.so --algo 1 --mod 8PSK --rate 1/2 --batch 262144 --rounds 4 > $O/ab_lmw4.txt 2>&1 || exit 1
