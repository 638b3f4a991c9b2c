set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r02pl
mkdir -p $O
timeout -k 10 120 python tools/placement_counters.py --handles 8 --rounds 2 > $O/plain.txt
P="timeout -s KILL 150 rocprofv3"
$P --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $O/utcl1 -o u --output-format csv -- python tools/placement_counters.py --rounds 1 > $O/utcl1.txt
$P --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum -d $O/tcc -o t --output-format csv -- python tools/placement_counters.py --rounds 1 > $O/tcc.txt
$P --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum -d $O/lat -o l --output-format csv -- python tools/placement_counters.py --rounds 1 > $O/lat.txt
