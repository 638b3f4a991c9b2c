set -euo pipefail
O=gpurun_out/${TAG:-r02cfg}
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu --mod QPSK --n 212 --batch 102400 --steps 10 > $O/c1_qpsk212.json 2> $O/c1.err
timeout -k 10 300 python bench.py --no-cpu --mod 8PSK --rate 1/2 --algo log-map --batch 1048576 --steps 3 --warmup 1 > $O/c3_8psk_logmap.json 2> $O/c3.err
timeout -k 10 300 python bench.py --no-cpu --mod 256QAM --batch 1048576 --steps 3 --warmup 1 > $O/c4_256qam.json 2> $O/c4.err
timeout -k 10 300 python -m modulations_amd.ber --mod 256QAM --n 752 --rate 1/3 --ebn0=-2:10:4 --codewords 1000000 --batch 262144 --out $O/c4_ber_sweep.json > $O/c4_ber.log 2>&1
