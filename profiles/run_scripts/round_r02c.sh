# Round-2 checkpoint: full GPU test suite, smoke, headline bench, and the rocprof passes of the bench.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-r02c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tools/profile.sh $TAG python bench.py --steps 2 --warmup 1 --no-cpu
