# Shortest segment (TDEC_FR_LMIN 16 / 24 / 32 / 48) now that small N runs one wave per
# direction (rounds inside the wave, no cross-wave barriers): frame parity under the
# shortest floor, then per-call latencies at N = 48 / 64 / 212, two passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
TDEC_LIB_VARIANT=l16 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py tests/test_siso_f64.py tests/test_gpu_logmap.py > $O/tests_l16.log 2>&1 || exit 1
for pass in 1 2; do
for v in base l16 l24 l32; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "64 1/3" "212 1/3"; do
    set -- $nr
    LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_$pass.json 2>&1 || exit 1
  done
done
done
unset TDEC_LIB_VARIANT
