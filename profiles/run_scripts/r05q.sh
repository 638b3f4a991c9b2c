# Counters of k_demap_planes alone (16QAM, 1 M codewords, the current library)
set -o pipefail
export TMPDIR=/tmp
tools/profile.sh r05q python tools/ab_demap.py modulations_amd/lib/libtdec.so --rounds 1
