# Round 5: kernel durations of the per-call paths (SISO and decode() per frame) under rocprofv3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o calls -- python tools/call_probe.py > $O/probe.log 2>&1 || exit 1
