#!/bin/bash
# configs[1] (QPSK N=212 r=1/3) decode time against batch size: is the 100 k
# point bound by one tile's latency (fewer tiles than wave slots) or by HBM?
set -o pipefail
mkdir -p gpurun_out/bsweep
for B in ${BATCHES:-25600 51200 102400 131072 163840 204800 262144}; do
  timeout -k 10 120 python -u bench.py --mod QPSK --n 212 --batch $B --steps 10 --no-cpu \
    > gpurun_out/bsweep/b$B.json 2> gpurun_out/bsweep/b$B.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bsweep/b$B.json'));print($B, round(d['decode_kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,3))"
done
