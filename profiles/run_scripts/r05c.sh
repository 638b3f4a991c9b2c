# Round 5: A/B of the frame decoder's minimum segment length (TDEC_FR_LMIN) on the
# per-call paths: SISO call and decode() per frame at N = 48 / 212 / 752, two passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
for pass in 1 2; do
for v in base lmin32 lmin48 lmin64 lmin96; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/siso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "212 1/3" "752 1/2"; do
    set -- $nr
    LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lat_${v}_$1_$pass.json 2>&1 || exit 1
  done
done
done
