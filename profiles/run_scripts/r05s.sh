# Tail gate (tdec_tail_gate): batch i+1's demap released into the slots batch i's
# decoder waves free as they retire.  The overlapped-pipeline parity test, then
# bench.py serial vs --overlap alternating, 3 processes each (configs[2]).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_workload.py > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 > $O/serial_$r.json 2> $O/serial_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --overlap > $O/overlap_$r.json 2> $O/overlap_$r.err || exit 1
done
