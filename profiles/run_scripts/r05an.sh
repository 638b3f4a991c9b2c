# Demapper structure A/B: planar LDS tile (pl), persistent blocks with the end-of-item
# barrier not waiting for the plane stores (pnv), both (plpnv); 16QAM / 256QAM / QPSK.
# Parity of the combined variant first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05an
mkdir -p $O
TDEC_LIB_VARIANT=plpnv timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_nonfinite.py tests/test_gpu_workload.py > $O/tests_plpnv.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "256QAM" "QPSK --n 212"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_pl.so $L/libtdec_pnv.so $L/libtdec_plpnv.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_plpnv.so $L/libtdec_pnv.so $L/libtdec_pl.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
