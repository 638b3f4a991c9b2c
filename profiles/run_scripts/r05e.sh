# Round 5: log-MAP in the frame decoder / frame SISO: tests and per-call latency.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_logmap.py tests/test_gpu_parity.py tests/test_hypothesis_gpu.py tests/test_logmap_accuracy.py > $O/tests.log 2>&1 || exit 1
for nr in "48 1/3" "212 1/3" "752 1/2" "848 1/3"; do
  set -- $nr
  LAT_ALGO=log-map LAT_BATCHES=1,64,1024,4096 timeout -k 10 300 python tools/latency.py $1 $2 > $O/lat_lm_$1.json 2>&1 || exit 1
done
TDEC_LOWLAT_MAX=0 LAT_ALGO=log-map LAT_BATCHES=64,1024,4096,8192 timeout -k 10 300 python tools/latency.py 752 1/2 > $O/lat_lm_tp_752.json 2>&1 || exit 1
LAT_ALGO=log-map LAT_BATCHES=8192 TDEC_LOWLAT_MAX=8192 timeout -k 10 300 python tools/latency.py 752 1/2 > $O/lat_lm_fr8192_752.json 2>&1 || exit 1
