# Demapper third pass: 16QAM's closed-form search with one range test per symbol
# (sym_llrs_pairs16): exactness self-tests + demap parity (new arithmetic-variant
# cases), then A/B against the round-4 kernels (dm0), both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_modem.py \
  tests/test_nonfinite.py tests/test_gpu_workload.py > $O/tests.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "QPSK --n 212" "8PSK --rate 1/2"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_dm0.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_dm0.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
