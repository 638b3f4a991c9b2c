# Round 6: configs[4] as the sweep it is: 256QAM, N = 752 r = 1/3,
# 8 iterations max-log, Eb/N0 -2..10 dB in 1 dB steps, 1 048 576 codewords per point
# (one batch), reference interleaver (and the true permutation for comparison); then
# the bench line + rocprof kernel trace and PMC passes at both ends of the sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
for il in reference valid-perm; do
  timeout -k 10 600 python -u -m modulations_amd.ber --mod 256QAM --n 752 --rate 1/3 --ebn0=-2:10:1 \
    --codewords 1048576 --batch 1048576 --interleaver $il --out $O/c4_sweep_$il.json > $O/c4_sweep_$il.log 2>&1 || exit 1
done
for e in -2 10; do
  ./tools/prof_config.sh r06c/c4_ebn0_$e --mod 256QAM --batch 1048576 --steps 3 --warmup 1 --ebn0=$e || exit 1
done
echo r06c done
