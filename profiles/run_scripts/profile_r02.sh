# Round-2 headline profile: bench + kernel trace + FETCH/WRITE + SQ passes of the same command
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-r02b}
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tools/profile.sh $TAG python bench.py --steps 2 --warmup 1 --no-cpu
