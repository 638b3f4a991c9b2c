# Round 5, first GPU pass: the new float64 SISO tests, the N = 848 frame decoder and
# the full GPU suite, smoke, per-call latencies (SISO f32 / f64 and the C call alone;
# decode() per frame at N = 48 / 212 / 752 / 848 and log-MAP), the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_siso_f64.py tests/test_gpu_frame.py > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
for nr in "48 1/3" "212 1/3" "752 1/2" "848 1/3"; do
  set -- $nr
  LAT_BATCHES=1,64,1024 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_$1.json 2>&1 || exit 1
done
LAT_ALGO=log-map LAT_BATCHES=1,64 timeout -k 10 300 python tools/latency.py 752 1/2 > $O/lat_logmap_752.json 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
