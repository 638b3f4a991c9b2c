# Final library on a second box: the default bench line three times (the r05y5 box ran
# the unchanged decoder at 237.9 ms per 1 M codewords, 7 % slower than any box before).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y5b
mkdir -p $O
rocm-smi --showclocks --showpower --showtemp > $O/smi.txt 2>&1 || true
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
