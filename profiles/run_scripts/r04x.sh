set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04x
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lowlat.py > gpurun_out/r04x/tests.log 2>&1 || exit 1
