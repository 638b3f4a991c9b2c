# Demapper wave-private variant (TDEC_DM_WAVE: each wave owns 16 codewords of the tile,
# no block barrier between the phases; wvk12: with 12 couples per block): parity of wv
# first, then in-process A/B against the default, both orders, five tables.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ap
mkdir -p $O
TDEC_LIB_VARIANT=wv timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_nonfinite.py tests/test_gpu_workload.py > $O/tests_wv.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "256QAM" "64QAM" "8PSK" "QPSK --n 212"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_wv.so $L/libtdec_wvk12.so --mod $m --rounds 9 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_wvk12.so $L/libtdec_wv.so $L/libtdec.so --mod $m --rounds 9 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
