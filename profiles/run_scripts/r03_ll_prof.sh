#!/bin/bash
# Where a decode() call's 3.7 ms go: rocprofv3 kernel trace of tools/latency.py
# (per-kernel time of k_turbo_decode_lowlat / k_depuncture against the host-measured call).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r03llp}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/kt -o run -- python tools/latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
find $O/kt -name '*kernel_stats.csv' -exec cat {} \;
find $O/kt -name '*memory_copy_stats.csv' -exec cat {} \;
