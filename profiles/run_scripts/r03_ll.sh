#!/bin/bash
# low-latency decoder: GPU tests + per-call latency (tools/latency.py)
set -o pipefail
O=gpurun_out/${TAG:-r03ak}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowlat.py -x -q --timeout 120 --timeout-method thread > $O/ll_tests.log 2>&1 || { tail -30 $O/ll_tests.log; exit 1; }
tail -1 $O/ll_tests.log
timeout -k 10 200 python tools/latency.py > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.json
