set -o pipefail
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
O=gpurun_out/r04k
L=modulations_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_demap_split.py tests/test_nonfinite.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || exit 1
for m in 256QAM 64QAM 16QAM; do timeout -k 10 200 python tools/ab_demap.py $L/libtdec_nosplit.so $L/libtdec.so --mod $m --rounds 5 > $O/ab_demap_$m.txt 2>&1 || exit 1; done
for m in 256QAM 16QAM; do timeout -k 10 200 python tools/ab_demap.py $L/libtdec.so $L/libtdec_nosplit.so --mod $m --rounds 5 > $O/ab_demap_${m}_rev.txt 2>&1 || exit 1; done
