# Round 6, first pass on the pruned library (knobs removed, ADVICE r5 fixes,
# sub-tile units): the GPU suite, smoke, the default bench line, in-process A/B
# against the round-5 library (lib/libtdec_r05.so) on configs [2], [1] and [3], the
# sub-tile A/B at configs[1] (lib/libtdec_nosub.so), and the wave-timing builds'
# per-wave shader clock at configs [2], [1] and [3] (DVFS).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
L=modulations_amd/lib
timeout -k 10 300 python tools/ab.py $L/libtdec_r05.so $L/libtdec.so --rounds 4 > $O/ab_c2.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_r05.so --rounds 4 > $O/ab_c2_rev.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_r05.so $L/libtdec_nosub.so $L/libtdec.so --n 212 --mod QPSK --batch 102400 --rounds 8 > $O/ab_c1.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_nosub.so $L/libtdec_r05.so --n 212 --mod QPSK --batch 102400 --rounds 8 > $O/ab_c1_rev.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_r05.so $L/libtdec.so --n 752 --rate 1/2 --mod 8PSK --algo 1 --rounds 3 > $O/ab_c3.txt 2>&1 || exit 1
TDEC_WAVE_DUMP=$O/wd_c2.txt timeout -k 10 300 python tools/wave_dump.py $L/libtdec_wt.so --n 752 --mod 16QAM --batch 1048576 > $O/wave_c2.txt 2>&1 || exit 1
TDEC_WAVE_DUMP=$O/wd_c1.txt timeout -k 10 300 python tools/wave_dump.py $L/libtdec_wtnosub.so $L/libtdec_wt.so > $O/wave_c1.txt 2>&1 || exit 1
TDEC_WAVE_DUMP=$O/wd_c3.txt timeout -k 10 300 python tools/wave_dump.py $L/libtdec_wt.so --n 752 --rate 1/2 --mod 8PSK --algo 1 --batch 262144 > $O/wave_c3.txt 2>&1 || exit 1
rm -f $O/wd_*.txt
echo r06a done
