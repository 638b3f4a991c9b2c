#!/bin/bash
# Round-3 evidence for every BASELINE config line: bench JSON + rocprof kernel trace / PMC passes
# (tools/prof_config.sh), then the configs[4] Eb/N0 sweeps (13 points x 10 M codewords, both interleavers).
#   TAG=r03x tools/configs.sh [c1] [c3] [c4] [sweep]
set -o pipefail
T=${TAG:-r03cfg}
for what in "$@"; do
  case $what in
    c1) ./tools/prof_config.sh ${T}_c1 --mod QPSK --n 212 --batch 102400 --steps 10 || exit $? ;;
    c2) ./tools/prof_config.sh ${T}_c2 --steps 5 || exit $? ;;
    c3) ./tools/prof_config.sh ${T}_c3 --mod 8PSK --rate 1/2 --algo log-map --batch 1048576 --steps 3 --warmup 1 || exit $? ;;
    c4) ./tools/prof_config.sh ${T}_c4 --mod 256QAM --batch 1048576 --steps 3 --warmup 1 || exit $? ;;
    sweep)
      mkdir -p gpurun_out/${T}_sweep
      for il in reference valid-perm; do
        timeout -k 10 600 python -u -m modulations_amd.ber --mod 256QAM --n 752 --rate 1/3 --ebn0=-2:10:1 \
          --codewords 10000000 --batch 1048576 --interleaver $il --out gpurun_out/${T}_sweep/c4_${il}.json \
          > gpurun_out/${T}_sweep/c4_${il}.log 2>&1 || exit $?
      done ;;
  esac
done
