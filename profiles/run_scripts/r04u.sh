set -o pipefail
mkdir -p gpurun_out/r04u
export TMPDIR=/tmp
O=gpurun_out/r04u
LAT_BATCHES=1024,2048,4096,8192,16384,32768 TDEC_LOWLAT_MAX=0 timeout -k 10 300 python tools/latency.py 752 1/2 > $O/lat_throughput.json 2>&1 || exit 1
LAT_BATCHES=1024,2048,4096,8192,16384,32768 TDEC_LOWLAT_MAX=65536 timeout -k 10 300 python tools/latency.py 752 1/2 > $O/lat_frame.json 2>&1 || exit 1
LAT_BATCHES=1024,4096,8192,16384,32768 TDEC_LOWLAT_MAX=0 timeout -k 10 300 python tools/latency.py 212 1/3 > $O/lat212_throughput.json 2>&1 || exit 1
LAT_BATCHES=1024,4096,8192,16384,32768 TDEC_LOWLAT_MAX=65536 timeout -k 10 300 python tools/latency.py 212 1/3 > $O/lat212_frame.json 2>&1 || exit 1
