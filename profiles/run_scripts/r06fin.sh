# Round 6, the one final evidence pass on the final library:
# the full GPU suite, smoke, the default bench line, per-call latencies, and bench
# line + rocprof kernel trace + PMC passes of every BASELINE config (traffic.json is
# stamped from these with this library).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06fin
mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
TAG=r06fin tools/configs.sh c1 c2 c3 c4 || exit 1
echo r06fin done
