# Frame recursion phase timers (TDEC_FR_STATS=2 build, two waves per direction at
# N = 752; one codeword per call and 64): wave 0's phase A per SISO -> ns per step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ak
mkdir -p $O
for B in 1 64; do
  FRSTATS_VARIANT=frtime timeout -k 10 120 python tools/frame_stats.py 752 1/3 2.0 $B > $O/frtime_752_$B.json 2>&1 || exit 1
done
