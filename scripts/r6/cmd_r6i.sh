export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
T=none,none,none,none,none,none,none,none,none,none
FLS_PLACEMENT_GOOD=0 timeout -k 10 300 python3 -u scripts/placement_probe.py --rounds 4 --trials $T > $O/placement_q1_r6j.txt 2>&1 || exit 2
timeout -k 10 300 python3 -u scripts/placement_probe.py --rounds 4 --trials $T > $O/placement_q4_r6j.txt 2>&1 || exit 3
timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 100 --rounds 3 --trials none,none,none > $O/placement_q4_sf100_r6j.txt 2>&1 || exit 4
