# Round 6, experiments, all in-process A/B + rocprof:
#  - configs[2]: discarded P1 / Le1 stores as dropped buffer stores (oor), the last
#    backward window without its self re-read (lastw), both (oorlw);
#  - configs[3]: the log-MAP max* correction from an LDS table (lut, timing only:
#    different bits);
#  - kernel trace + PMC passes (bytes, VALU / wait counters, GRBM clock) per variant;
#  - the tests new this round (one-round batches, 4 096-row log-MAP oracle check).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
L=modulations_amd/lib
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_properties.py tests/test_gpu_logmap.py tests/test_siso_f64.py > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_oor.so $L/libtdec_lastw.so $L/libtdec_oorlw.so --rounds 5 > $O/ab_c2.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_oorlw.so $L/libtdec_lastw.so $L/libtdec_oor.so $L/libtdec.so --rounds 5 > $O/ab_c2_rev.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec.so $L/libtdec_lut.so --n 752 --rate 1/2 --mod 8PSK --algo 1 --rounds 3 > $O/ab_c3.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab.py $L/libtdec_lut.so $L/libtdec.so --n 752 --rate 1/2 --mod 8PSK --algo 1 --rounds 3 > $O/ab_c3_rev.txt 2>&1 || exit 1
for v in base oor lastw; do
  lib=$L/libtdec.so; [ $v = base ] || lib=$L/libtdec_$v.so
  tools/profile.sh r06b/prof_c2_$v python tools/ab.py $lib --rounds 1 > $O/prof_c2_$v.log 2>&1 || exit 1
done
for v in base lut; do
  lib=$L/libtdec.so; [ $v = base ] || lib=$L/libtdec_$v.so
  tools/profile.sh r06b/prof_c3_$v python tools/ab.py $lib --rounds 1 --n 752 --rate 1/2 --mod 8PSK --algo 1 > $O/prof_c3_$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/prof_c3_${v}_lds -o l --output-format csv -- python tools/ab.py $lib --rounds 1 --n 752 --rate 1/2 --mod 8PSK --algo 1 > $O/prof_c3_${v}_lds.log 2>&1 || true
done
echo r06b done
