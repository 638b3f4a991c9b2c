#!/bin/bash
# Build libtdec.so from the sources of a git revision (for in-process A/B with tools/ab.py):
#   tools/build_rev.sh <rev> <name> [-DDEFINE ...]  ->  modulations_amd/lib/libtdec_<name>.so
set -euo pipefail
rev=$1; name=$2; shift 2
d=$(mktemp -d)
mkdir -p $d/csrc $d/include
for f in tdec_api.hip tdec_kernels.hip tdec_workload.hip tdec_spl.hip tdec_lowlat.hip tdec_frame.hip npmath.hip; do
  git show $rev:modulations_amd/csrc/$f > $d/csrc/$f 2>/dev/null || rm -f $d/csrc/$f
done
git show $rev:include/tdec.h > $d/include/tdec.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fno-gpu-flush-denormals-to-zero -w "$@" -I $d/include -o modulations_amd/lib/libtdec_$name.so $d/csrc/tdec_api.hip
rm -rf $d
echo modulations_amd/lib/libtdec_$name.so
