# (1) the multi-rank bench path on real GPU memory: 2 ranks on GPU 0 over gloo
#     (the driver's N > 1 launch shape, rehearsed on a 1-GPU box);
# (2) frame vs throughput decoder crossover after round 5's frame speedups:
#     decode_batch at B = 2048 .. 16384, default routing vs TDEC_LOWLAT_MAX=0
#     (throughput decoder) vs TDEC_LOWLAT_MAX=16384 (frame decoder), N = 212 / 752.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 2 --all-on-device0 --dist-backend gloo --steps 3 --warmup 1 --batch 65536 --no-cpu > $O/bench_2ranks.json 2> $O/bench_2ranks.err || exit 1
for n in "212 1/3" "752 1/3"; do
  set -- $n
  for v in default thr frame; do
    case $v in default) unset TDEC_LOWLAT_MAX ;; thr) export TDEC_LOWLAT_MAX=0 ;; frame) export TDEC_LOWLAT_MAX=16384 ;; esac
    LAT_BATCHES=2048,4096,8192,12288,16384 timeout -k 10 300 python tools/latency.py $1 $2 > $O/x_${v}_$1.json 2>&1 || exit 1
  done
done
unset TDEC_LOWLAT_MAX
