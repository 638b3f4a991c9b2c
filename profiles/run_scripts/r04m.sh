set -o pipefail
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
O=gpurun_out/r04m
L=modulations_amd/lib
TDEC_LIB_VARIANT=wpd4 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_nonfinite.py > $O/tests_wpd4.log 2>&1 || exit 1
for B in 1 64 1024; do timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_wpd4.so --batch $B --rounds 8 --mod QPSK --rate 1/2 > $O/ab_wpd4_$B.txt 2>&1 || exit 1; done
for v in frtime frtime4; do FRSTATS_VARIANT=$v timeout -k 10 120 python tools/frame_stats.py 752 1/2 2.0 1 > $O/${v}.json 2>&1 || exit 1; done
TDEC_LIB_VARIANT=wpd4 timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat_wpd4.json 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
