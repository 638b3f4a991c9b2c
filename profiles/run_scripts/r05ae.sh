# log-MAP: frame vs throughput decoder crossover after the 8-step log-MAP frame blocks
# (host-pointer decode_batch, N = 752 r = 1/2 and N = 212 r = 1/3).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ae
mkdir -p $O
export LAT_ALGO=log-map
for n in "752 1/2" "212 1/3"; do
  set -- $n
  for v in default thr frame; do
    case $v in default) unset TDEC_LOWLAT_MAX ;; thr) export TDEC_LOWLAT_MAX=0 ;; frame) export TDEC_LOWLAT_MAX=16384 ;; esac
    LAT_BATCHES=4096,6144,8192,12288 timeout -k 10 300 python tools/latency.py $1 $2 > $O/x_${v}_$1.json 2>&1 || exit 1
  done
done
