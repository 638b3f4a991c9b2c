# Workspace placement: does remapping the same physical chunks in other orders move
# the decode time?  4 fresh processes with 8 orders probed (printed), each then
# decoding 1 M codewords on the order it kept; 4 with the default single order.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
for r in 1 2 3 4; do
  TDEC_VMM_ORDERS=8 TDEC_PROBE_VERBOSE=1 timeout -k 10 200 python -u tools/vmm_orders.py > $O/k8_$r.txt 2>&1 || exit 1
  timeout -k 10 200 python -u tools/vmm_orders.py > $O/k1_$r.txt 2>&1 || exit 1
done
