# Validation of the round's last per-call / demap changes against "prev" (scan range
# test off, 16 couples per QPSK demap block, 4-step log-MAP frame blocks) and, by
# environment, one wave per recursion direction off (TDEC_FR_WPD1_MAX=0,
# TDEC_FR_SISO_WPD1_MAX=0): the GPU suites touching them, then per-call latencies
# (N = 48 / 64 / 212 / 220 / 424 / 752 / 848) and the QPSK / 8PSK demap A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py \
  tests/test_siso_f64.py tests/test_gpu_logmap.py tests/test_gpu_lowlat.py tests/test_nonfinite.py tests/test_gpu_parity.py \
  tests/test_gpu_selftest.py tests/test_gpu_demap_split.py tests/test_gpu_modem.py tests/test_gpu_workload.py \
  tests/test_hypothesis_gpu.py > $O/tests.log 2>&1 || exit 1
TDEC_FR_WPD1_MAX=0 TDEC_FR_SISO_WPD1_MAX=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py tests/test_siso_f64.py > $O/tests_wpd2.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "QPSK --n 212" "8PSK --rate 1/2"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_prev.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_prev.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
for pass in 1 2; do
for v in base wpd2; do
  if [ $v = wpd2 ]; then export TDEC_FR_WPD1_MAX=0 TDEC_FR_SISO_WPD1_MAX=0; else unset TDEC_FR_WPD1_MAX TDEC_FR_SISO_WPD1_MAX; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "64 1/3" "212 1/3" "220 1/3" "424 1/3" "752 1/3" "848 1/3"; do
    set -- $nr
    LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_$pass.json 2>&1 || exit 1
  done
  LAT_ALGO=log-map LAT_BATCHES=1 timeout -k 10 200 python tools/latency.py 752 1/2 > $O/lmlat_${v}_752_$pass.json 2>&1 || exit 1
done
done
unset TDEC_FR_WPD1_MAX TDEC_FR_SISO_WPD1_MAX
