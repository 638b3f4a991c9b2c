set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r02cal
timeout -k 10 60 tools/mb/fetch_cal > gpurun_out/r02cal/plain.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02cal/f -o f --output-format csv -- tools/mb/fetch_cal > /dev/null
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02cal/w -o w --output-format csv -- tools/mb/fetch_cal > /dev/null
tools/profile.sh r02a python bench.py --steps 2 --warmup 1 --no-cpu
