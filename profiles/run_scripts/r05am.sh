# Demapper time split (timing build dmexp = TDEC_DM_EXP=1: phase 1 without the demap
# arithmetic, wrong planes): 16QAM and QPSK.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am
mkdir -p $O
L=modulations_amd/lib
for m in "16QAM" "QPSK --n 212"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab_demap.py $L/libtdec.so $L/libtdec_dmexp.so --mod $m --rounds 7 > $O/ab_${tag}.txt 2>&1 || exit 1
done
