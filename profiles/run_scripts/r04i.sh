set -o pipefail
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
O=gpurun_out/r04i
for v in frtime frexp1 frexp2 frexp3 frexp4; do FRSTATS_VARIANT=$v timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 1 > $O/${v}.json 2>&1 || exit 1; done
