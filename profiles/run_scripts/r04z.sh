set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
for i in 1 2; do
TDEC_ZC=0 LAT_BATCHES=1,16,64,256 timeout -k 10 200 python tools/latency.py 752 1/2 > $O/lat_dma_$i.json 2>&1 || exit 1
LAT_BATCHES=1,16,64,256 timeout -k 10 200 python tools/latency.py 752 1/2 > $O/lat_zc_$i.json 2>&1 || exit 1
TDEC_ZC=0 timeout -k 10 120 python tools/siso_lat.py > $O/siso_dma_$i.json 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_zc_$i.json 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
TAG=r04z tools/configs.sh c2 c4 || exit 1
