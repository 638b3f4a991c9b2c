#!/bin/bash
# Low-latency SISO boundary: GPU suite, then bcjr_max_log_map per-call ms with and without it.
set -o pipefail
O=gpurun_out/${TAG:-r03sisoll}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for m in 0 default; do
  if [ $m = 0 ]; then export TDEC_LOWLAT_MAX=0; else unset TDEC_LOWLAT_MAX; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat_$m.json 2> $O/siso_lat_$m.err || { tail $O/siso_lat_$m.err; exit 1; }
  cat $O/siso_lat_$m.json
done
