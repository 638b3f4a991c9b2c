set -o pipefail
mkdir -p gpurun_out/r04s
export TMPDIR=/tmp
O=gpurun_out/r04s
L=modulations_amd/lib
TDEC_LIB_VARIANT=asmblk timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_nonfinite.py > $O/tests_asmblk.log 2>&1 || exit 1
for B in 1 64 1024; do timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_asmblk.so --batch $B --rounds 8 --mod QPSK --rate 1/2 > $O/ab_asmblk_$B.txt 2>&1 || exit 1; done
TDEC_LIB_VARIANT=asmblk timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat_asmblk.json 2>&1 || exit 1
