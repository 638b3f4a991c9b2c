# Gray search (64 / 256QAM) with the differences it formed and one range test per
# symbol for the unscaled sequences (TDEC_DM_GRAYPRE): demap parity + self-tests,
# then A/B against gp0 (the round-5 library before it), both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_modem.py tests/test_nonfinite.py \
  tests/test_gpu_workload.py > $O/tests.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "256QAM" "64QAM"; do
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_gp0.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${m}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_gp0.so --mod $m --rounds 7 > $O/ab_${m}_b.txt 2>&1 || exit 1
done
