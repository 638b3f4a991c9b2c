# Placement study: physically contiguous workspace (TDEC_WS_ALLOC=contiguous) with a
# swept padding after each workspace row (TDEC_ROW_PAD lanes of 16 B).
set -euo pipefail
O=gpurun_out/r02pp
mkdir -p $O
for pad in ${PADS:-0 16 64 256 1024 4096 32768 65536}; do
  TDEC_ROW_PAD=$pad TDEC_WS_ALLOC=contiguous timeout -k 10 120 python tools/placement_counters.py --handles 3 --rounds 2 > $O/contig_pad$pad.txt 2>&1
done
