# Demapper occupancy A/B: the f64 split kernels are register-bound at 3 (16 / 64QAM) and
# 2 (256QAM) waves per SIMD; TDEC_DM_WPE=4 / 3 caps their registers at 128 / 168.
# Parity of wpe4 first, then in-process A/B against the default, both orders.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aq
mkdir -p $O
TDEC_LIB_VARIANT=wpe4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_nonfinite.py tests/test_gpu_workload.py > $O/tests_wpe4.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "16QAM" "256QAM" "64QAM"; do
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_wpe4.so $L/libtdec_wpe3.so --mod $m --rounds 9 > $O/ab_${m}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_wpe3.so $L/libtdec_wpe4.so $L/libtdec.so --mod $m --rounds 9 > $O/ab_${m}_b.txt 2>&1 || exit 1
done
