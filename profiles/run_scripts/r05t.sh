# Frame decoder: 8-step fast blocks (TDEC_FR_BLK8) -- the frame / SISO parity
# suites, then A/B against the 4-step blocks (fr4) on the per-call paths (SISO call
# and decode() per frame at N = 48 / 212 / 752, batch 1 / 64 / 1024), two passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py \
  tests/test_siso_f64.py tests/test_gpu_logmap.py tests/test_gpu_lowlat.py tests/test_nonfinite.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
for pass in 1 2; do
for v in base fr4; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "212 1/3" "752 1/3" "752 1/2"; do
    set -- $nr
    LAT_BATCHES=1,64,1024 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_${2/\//}_$pass.json 2>&1 || exit 1
  done
done
done
