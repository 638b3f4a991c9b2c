# New frame tests: every SISO length 1..160 on both recursion layouts, the decoder on
# both layouts at every block size.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py -k "every_length or both_recursion" > $O/tests.log 2>&1 || exit 1
