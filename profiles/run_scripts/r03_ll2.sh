#!/bin/bash
# low-latency decoder with LDS-staged interleaver tables: GPU suite + per-call latency + kernel time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r03ll2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python tools/latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/latency.py > $O/latency_prof.json 2> $O/latency_prof.err || { tail $O/latency_prof.err; exit 1; }
find $O/kt -name '*kernel_stats.csv' -exec cat {} \;
