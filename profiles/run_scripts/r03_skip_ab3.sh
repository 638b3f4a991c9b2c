#!/bin/bash
# Dead-extrinsic skip, part 3: GPU suite on the library, log-MAP midpoint skip A/B
# (libtdec_prev.so = -DTDEC_SKIP_MID_LM=0 -DTDEC_LL_SKIP_UNUSED=0) and the
# low-latency decoder's per-call latency with / without the used-position list.
set -o pipefail
O=gpurun_out/${TAG:-r03sk3}; mkdir -p $O
L=modulations_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python tools/ab.py $L/libtdec_prev.so $L/libtdec.so --algo 1 --mod 8PSK --rate 1/2 --batch 262144 --rounds 3 > $O/ab_lm.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm.log
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_prev.so --algo 1 --mod 8PSK --rate 1/2 --batch 262144 --rounds 3 > $O/ab_lm_r.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_lm_r.log
for v in prev new; do
  if [ $v = prev ]; then export TDEC_LIB_VARIANT=prev; else unset TDEC_LIB_VARIANT; fi
  timeout -k 10 200 python tools/latency.py > $O/latency_$v.json 2> $O/latency_$v.err || { tail $O/latency_$v.err; exit 1; }
  echo "$v"; cat $O/latency_$v.json
done
