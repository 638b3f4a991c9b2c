# Even segment split with at least TDEC_FR_LMIN = 32 steps per segment (n48: 48):
# the frame / SISO / log-MAP parity suites, then per-call latencies, two passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py \
  tests/test_siso_f64.py tests/test_gpu_logmap.py tests/test_gpu_lowlat.py tests/test_nonfinite.py \
  tests/test_hypothesis_gpu.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
for pass in 1 2; do
for v in base n48; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "64 1/3" "212 1/3" "220 1/3" "424 1/3" "752 1/3" "848 1/3"; do
    set -- $nr
    LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_$pass.json 2>&1 || exit 1
  done
done
done
unset TDEC_LIB_VARIANT
