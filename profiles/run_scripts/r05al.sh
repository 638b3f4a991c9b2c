# The plane kernels' LLRs in f32 form (f32o = TDEC_DM_F32OUT=1): demap parity under
# the variant, then A/B against the library per BASELINE table, both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05al
mkdir -p $O
TDEC_LIB_VARIANT=f32o timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_modem.py tests/test_nonfinite.py \
  tests/test_gpu_workload.py tests/test_gpu_fused.py > $O/tests_f32o.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "256QAM" "QPSK --n 212" "8PSK --rate 1/2"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_f32o.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_f32o.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
