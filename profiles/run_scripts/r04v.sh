set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04v
O=gpurun_out/r04v
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_nonfinite.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || exit 1
for m in 256QAM 16QAM; do timeout -k 10 200 python tools/ab_demap.py modulations_amd/lib/libtdec.so --mod $m --rounds 5 > $O/demap_$m.txt 2>&1 || exit 1; done
bash profiles/run_scripts/r04u.sh || exit 1
