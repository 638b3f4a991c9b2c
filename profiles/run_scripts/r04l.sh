set -o pipefail
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
O=gpurun_out/r04l
L=modulations_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_nonfinite.py tests/test_gpu_lowlat.py > $O/tests.log 2>&1 || exit 1
for B in 1 64 1024; do timeout -k 10 200 python tools/ab.py $L/libtdec_prevfr.so $L/libtdec.so --batch $B --rounds 8 --mod QPSK --rate 1/2 > $O/ab_fr_$B.txt 2>&1 || exit 1; done
FRSTATS_VARIANT=frtime timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 1 > $O/frtime.json 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
LAT_BATCHES=1,64,1024 timeout -k 10 200 python tools/latency.py 752 1/2 > $O/lat.json 2>&1 || exit 1
