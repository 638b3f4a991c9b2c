set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r02spl
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k state_per_lane -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o ab --output-format csv -- python tools/ab_siso.py --batch 131072 > $O/ab.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $O/sq -o s --output-format csv -- python tools/ab_siso.py --batch 131072 --reps 1 > $O/ab_sq.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format csv -- python tools/ab_siso.py --batch 131072 --reps 1 > $O/ab_f.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w -o w --output-format csv -- python tools/ab_siso.py --batch 131072 --reps 1 > $O/ab_w.txt 2>&1
