set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python tools/prof_workload.py > gpurun_out/r02wl_plain.txt 2>&1
tools/profile.sh r02wl python tools/prof_workload.py
