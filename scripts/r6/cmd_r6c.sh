export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 120 ./scripts/membw6 > $O/membw6_r6c.txt 2>&1 || exit 1
T=none,pad:2,pad:64,pad:1024,none,none
timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $O/pl_pmc1_r6c -o pmc --output-format csv -- python3 -u scripts/placement_probe.py --trials $T > $O/placement_pmc1_r6c.txt 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum -d $O/pl_pmc2_r6c -o pmc --output-format csv -- python3 -u scripts/placement_probe.py --trials $T > $O/placement_pmc2_r6c.txt 2>&1 || exit 3
timeout -k 10 200 python3 -u scripts/placement_probe.py --trials $T > $O/placement_plain_r6c.txt 2>&1 || exit 4
python3 scripts/pmc_trials.py fused_kernel 22 $O/pl_pmc1_r6c > $O/pl_pmc1_trials_r6c.txt
python3 scripts/pmc_trials.py fused_kernel 22 $O/pl_pmc2_r6c > $O/pl_pmc2_trials_r6c.txt
