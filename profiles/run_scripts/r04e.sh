set -o pipefail
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
O=gpurun_out/r04e
L=modulations_amd/lib
timeout -k 10 60 python tools/hip_probe.py > $O/hip_probe.txt 2>&1
timeout -k 10 60 python tools/hip_probe.py --torch > $O/hip_probe_torch.txt 2>&1
timeout -k 10 120 python tools/frame_stats.py 752 1/3 2.0 64 > $O/stats752.json 2>&1 || exit 1
timeout -k 10 120 python tools/frame_stats.py 212 1/3 2.0 64 > $O/stats212.json 2>&1 || exit 1
timeout -k 10 120 python tools/merge_depth.py --n 212 --mod QPSK --batch 102400 > $O/merge_c1.txt 2>&1 || exit 1
timeout -k 10 120 python tools/merge_depth.py --n 752 --mod 16QAM --batch 262144 > $O/merge_c2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_rs1.so --n 212 --mod QPSK --batch 102400 --rounds 8 > $O/ab_rs1_c1.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_rs1.so --rounds 6 > $O/ab_rs1_c2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_ck16.so --n 212 --mod QPSK --batch 102400 --rounds 6 > $O/ab_ck16_c1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py $L/libtdec.so $L/libtdec_ck16.so --n 424 --rate 1/2 --mod QPSK --batch 65536 --rounds 2 > $O/ab_ck16_424.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec.so $L/libtdec_ck16.so --rounds 6 > $O/ab_ck16_c2.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $L/libtdec_ck16.so $L/libtdec.so --rounds 6 > $O/ab_ck16_c2_rev.txt 2>&1 || exit 1
LAT_BATCHES=1,64,1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o lat -- python tools/latency.py 752 1/2 > $O/lat_prof.json 2>&1 || exit 1
timeout -k 10 120 python tools/siso_lat.py > $O/siso_lat.json 2>&1 || exit 1
for m in 256QAM 64QAM 16QAM; do timeout -k 10 200 python tools/ab_demap.py $L/libtdec_dmold.so $L/libtdec.so --mod $m --rounds 5 > $O/ab_demap_$m.txt 2>&1 || exit 1; done
timeout -k 10 300 python tools/ab.py $L/libtdec_lmold.so $L/libtdec.so --algo 1 --mod 8PSK --rate 1/2 --batch 262144 --rounds 4 > $O/ab_lm.txt 2>&1 || exit 1
