set -o pipefail
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
O=gpurun_out/r04h
for B in 1 64; do FRSTATS_VARIANT=frtime timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 $B > $O/frtime_752_B$B.json 2>&1 || exit 1; done
FRSTATS_VARIANT=frtime timeout -k 10 120 python tools/frame_stats.py 212 1/3 2.0 1 > $O/frtime_212_B1.json 2>&1 || exit 1
