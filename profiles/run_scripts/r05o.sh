# Demapper: unscaled f32 / f64 division and square root (TDEC_DM_FAST64) and the
# one-ahead symbol prefetch (TDEC_DM_PF): the exactness self-test, the demap parity
# tests, then in-process A/B of k_demap_planes per BASELINE table (both orders).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_modem.py \
  tests/test_nonfinite.py tests/test_gpu_workload.py > $O/tests.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "QPSK --n 212" "8PSK --rate 1/2" "256QAM"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_dm0.so $L/libtdec_dmpf.so $L/libtdec_dmfast.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_dmfast.so $L/libtdec_dmpf.so $L/libtdec_dm0.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
