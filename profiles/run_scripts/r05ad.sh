# The raised frame-decoder batch limits (12 288 at N >= 400, 8 192 below): the frame /
# low-latency / lowlat-routing GPU tests, then the host-pointer batch sweep again.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py \
  tests/test_gpu_lowlat.py tests/test_gpu_properties.py > $O/tests.log 2>&1 || exit 1
for n in "212 1/3" "752 1/3"; do
  set -- $n
  LAT_BATCHES=4096,8192,12288,16384 timeout -k 10 300 python tools/latency.py $1 $2 > $O/x_default_$1.json 2>&1 || exit 1
done
