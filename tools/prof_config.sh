#!/bin/bash
# Round-3 profile of one bench configuration: bench line + kernel trace + PMC passes
#   tools/prof_config.sh <tag> <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=$1
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u bench.py --no-cpu "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
tools/profile.sh $TAG python bench.py --no-cpu --steps 1 --warmup 1 "$@"
