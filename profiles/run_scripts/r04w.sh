set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04w
O=gpurun_out/r04w
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
LAT_BATCHES=1,64,1024,8192 timeout -k 10 200 python tools/latency.py 752 1/2 > $O/lat.json 2>&1 || exit 1
TAG=r04w tools/configs.sh c2 c4 || exit 1
