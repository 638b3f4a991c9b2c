# Demapper instruction mix: the f64 VALU counters of k_demap_planes (16QAM, 1 M codewords,
# the bench's table dtype), to price its issue in cycles (f64 ops at 16 lanes per clock).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05at
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_INSTS_VALU[A-Z0-9_]*" $O/avail.txt | sort -u > $O/valu_counters.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 \
  -d $O/f64 -o p --output-format csv -- python tools/ab_demap.py modulations_amd/lib/libtdec.so --mod 16QAM --rounds 1 > $O/run.log 2>&1 || exit 1
