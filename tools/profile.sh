#!/bin/bash
# Kernel trace + PMC passes (separate runs, as MI355X_MICROARCH.md prescribes) of one command.
#   tools/profile.sh <outdir under gpurun_out> <command...>
# then: python tools/prof_summary.py gpurun_out/<outdir> profiles/<name> <codewords per launch>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/$1
shift
P="timeout -k 10 300 rocprofv3"
$P --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- "$@"
$P --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- "$@"
$P --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- "$@"
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o s --output-format csv -- "$@"
$P --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d $OUT/tcc -o t --output-format csv -- "$@"
