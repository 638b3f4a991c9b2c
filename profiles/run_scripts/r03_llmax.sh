#!/bin/bash
# Crossover of the low-latency decoder against the throughput decoder: per-call ms at
# B = 1024 .. 8192 with TDEC_LOWLAT_MAX = 0 (throughput decoder only) and 8192 (low-latency).
set -o pipefail
O=gpurun_out/${TAG:-r03llmax}; mkdir -p $O
for m in 0 8192; do
  TDEC_LOWLAT_MAX=$m LAT_BATCHES=512,1024,1536,2048,3072,4096,8192 timeout -k 10 300 python tools/latency.py > $O/lat_$m.json 2> $O/lat_$m.err || { tail $O/lat_$m.err; exit 1; }
  cat $O/lat_$m.json
done
