#!/bin/bash
set -o pipefail
O=gpurun_out/r03ai; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_workload.py -x -v --timeout 300 --timeout-method thread > $O/workload_tests.log 2>&1 || { tail -40 $O/workload_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/workload_tests.log | tail -15
