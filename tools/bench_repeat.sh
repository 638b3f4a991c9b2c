# Fresh-process repeatability of the headline bench (placement probe verbose).
#   tools/bench_repeat.sh <tag> <runs> [extra bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=$1; RUNS=$2; shift 2
mkdir -p gpurun_out/$TAG
for i in $(seq 1 $RUNS); do
  TDEC_PROBE_VERBOSE=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu "$@" \
    > gpurun_out/$TAG/run$i.json 2> gpurun_out/$TAG/run$i.err
  grep -h "decode kernel" gpurun_out/$TAG/run$i.err
done
