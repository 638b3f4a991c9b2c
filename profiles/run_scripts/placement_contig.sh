# Placement A/B: default hipMalloc workspaces vs one physically contiguous range (TDEC_WS_ALLOC=contiguous),
# 8 handles per fresh process, probe off.
set -euo pipefail
O=gpurun_out/r02pc
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python tools/placement_counters.py --handles 6 --rounds 2 > $O/default_$i.txt 2>&1
  TDEC_WS_ALLOC=contiguous timeout -k 10 150 python tools/placement_counters.py --handles 6 --rounds 2 > $O/contig_$i.txt 2>&1
done
