# rocprof passes (trace, FETCH, WRITE, SQ) of tools/ab.py on one library variant each.
#   tools/prof_ab_r02.sh <tag> lib1.so [lib2.so ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=$1; shift
for L in "$@"; do
  n=$(basename $L .so)
  tools/profile.sh ${TAG}_$n python tools/ab.py $L --rounds 1
done
