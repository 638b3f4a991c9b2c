set -o pipefail
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
O=gpurun_out/r04g
L=modulations_amd/lib
for m in 256QAM 64QAM 16QAM; do timeout -k 10 200 python tools/ab_demap.py $L/libtdec.so $L/libtdec_dmstats.so --mod $m --rounds 3 > $O/dm_stats_$m.txt 2>&1 || exit 1; done
for v in frtime frtime1; do for B in 1 64; do FRSTATS_VARIANT=$v timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 $B > $O/${v}_752_B$B.json 2>&1 || exit 1; done; done
FRSTATS_VARIANT=frtime timeout -k 10 120 python tools/frame_stats.py 212 1/3 2.0 1 > $O/frtime_212_B1.json 2>&1 || exit 1
FRSTATS_VARIANT=frstats timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 64 > $O/frstats_752_B64.json 2>&1 || exit 1
