# Demapper planar LDS tile (pl) against the default, two-way only (the r05an four-way
# runs showed a position effect after the persistent variants); both orders, five tables.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
L=modulations_amd/lib
for m in "16QAM" "256QAM" "64QAM" "8PSK" "QPSK --n 212"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_pl.so --mod $m --rounds 11 > $O/ab_${tag}_a.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec_pl.so $L/libtdec.so --mod $m --rounds 11 > $O/ab_${tag}_b.txt 2>&1 || exit 1
done
