# Four waves per recursion direction above N = 424 (w4 = TDEC_FR_WPD=4: 16 segments)
# against two, with the 8-step blocks: frame parity, then decode() per frame / B = 64.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
TDEC_LIB_VARIANT=w4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py > $O/tests_w4.log 2>&1 || exit 1
for pass in 1 2; do
for v in base w4; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  for nr in "752 1/3" "752 1/2" "848 1/3"; do
    set -- $nr
    LAT_BATCHES=1,64,1024 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_${2/\//}_$pass.json 2>&1 || exit 1
  done
done
done
unset TDEC_LIB_VARIANT
