# log-MAP small-batch limit 7 168: the log-MAP GPU suite (frame vs throughput at 7 169 rows)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_logmap.py tests/test_build_hygiene.py > $O/tests.log 2>&1 || exit 1
