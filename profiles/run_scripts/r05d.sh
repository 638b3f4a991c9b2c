# Round 5: the per-call SISO with the completion-flag wait (TDEC_SPIN, default on) against
# the stream wait, and the frame tests / f64 SISO tests with the new segment floor.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_siso_f64.py tests/test_gpu_frame.py tests/test_nonfinite.py tests/test_gpu_lowlat.py > $O/tests.log 2>&1 || exit 1
for pass in 1 2; do
for sp in 1 0; do
  TDEC_SPIN=$sp timeout -k 10 120 python tools/siso_lat.py > $O/siso_spin${sp}_$pass.json 2>&1 || exit 1
done
done
for nr in "48 1/3" "212 1/3" "752 1/2" "848 1/3"; do
  set -- $nr
  LAT_BATCHES=1,64,1024 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_$1.json 2>&1 || exit 1
done
