set -o pipefail
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
O=gpurun_out/r04f
L=modulations_amd/lib
for m in 256QAM 64QAM 16QAM 8PSK QPSK; do timeout -k 10 200 python tools/ab_demap.py $L/libtdec_dmnp.so $L/libtdec.so $L/libtdec_dmlean.so --mod $m --rounds 5 > $O/ab_demap_$m.txt 2>&1 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
LAT_BATCHES=1,64,1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lat -o lat -- python tools/latency.py 752 1/2 > $O/lat.json 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
