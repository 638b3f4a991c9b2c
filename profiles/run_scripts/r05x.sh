# (1) BPSK / QPSK / 8PSK scan with one range test per symbol (TDEC_DM_SCANPRE):
#     demap parity + self-tests, A/B against the library without it (sp1 = with), both orders;
# (2) configs[1] serial vs --overlap (tail gate), alternating 3 + 3;
# (3) couples per demap block (TDEC_DM_KC 16 / 12 / 8): LDS tile vs blocks per CU;
# (4) the log-MAP frame path in 8-step blocks (TDEC_FR_BLK8_LM);
# (5) one wave per recursion direction (TDEC_FR_WPD=1) on the per-call paths.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py \
  tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_modem.py tests/test_nonfinite.py \
  tests/test_gpu_workload.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || exit 1
TDEC_LIB_VARIANT=sp1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py tests/test_gpu_demap_split.py tests/test_gpu_parity.py tests/test_gpu_modem.py tests/test_nonfinite.py tests/test_gpu_workload.py tests/test_gpu_fused.py > $O/tests_sp1.log 2>&1 || exit 1
L=modulations_amd/lib
for m in "QPSK --n 212" "8PSK --rate 1/2"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_sp1.so --mod $m --rounds 7 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_sp1.so $L/libtdec.so --mod $m --rounds 7 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --mod QPSK --n 212 --batch 102400 --steps 20 --warmup 3 > $O/c1_serial_$r.json 2> $O/c1_serial_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu --mod QPSK --n 212 --batch 102400 --steps 20 --warmup 3 --overlap > $O/c1_overlap_$r.json 2> $O/c1_overlap_$r.err || exit 1
done
for m in "16QAM" "QPSK --n 212"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_kc12.so $L/libtdec_kc8.so --mod $m --rounds 7 > $O/kc_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_kc8.so $L/libtdec_kc12.so $L/libtdec.so --mod $m --rounds 7 > $O/kc_${tag}_b.txt 2>&1 || exit 1
done
# (4) log-MAP frame path in 8-step blocks (lm8 = TDEC_FR_BLK8_LM=1): log-MAP parity, then decode() per frame A/B
TDEC_LIB_VARIANT=lm8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_logmap.py tests/test_gpu_frame.py > $O/tests_lm8.log 2>&1 || exit 1
for pass in 1 2; do
for v in base lm8; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  for nr in "48 1/3" "752 1/2"; do
    set -- $nr
    LAT_ALGO=log-map LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/lmlat_${v}_$1_$pass.json 2>&1 || exit 1
  done
done
done
unset TDEC_LIB_VARIANT
# (5) one wave per recursion direction (wpd1 = TDEC_FR_WPD=1: no cross-wave barriers) at small N
TDEC_LIB_VARIANT=wpd1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py > $O/tests_wpd1.log 2>&1 || exit 1
for pass in 1 2; do
for v in base wpd1; do
  if [ $v = base ]; then unset TDEC_LIB_VARIANT; else export TDEC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/siso_lat.py > $O/wsiso_${v}_$pass.json 2>&1 || exit 1
  for nr in "48 1/3" "212 1/3" "752 1/3"; do
    set -- $nr
    LAT_BATCHES=1,64 timeout -k 10 200 python tools/latency.py $1 $2 > $O/wlat_${v}_$1_$pass.json 2>&1 || exit 1
  done
done
done
unset TDEC_LIB_VARIANT
