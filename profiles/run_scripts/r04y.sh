set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04y
O=gpurun_out/r04y
TDEC_SISO_ZC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_nonfinite.py -k siso > $O/tests_zc.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat_dma_$i.json 2>&1 || exit 1
TDEC_SISO_ZC=1 timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat_zc_$i.json 2>&1 || exit 1
done
