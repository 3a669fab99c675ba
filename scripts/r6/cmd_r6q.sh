# placement rating vs decode time at SF25 and c3 (rate only: FLS_PLACEMENT_GOOD=0), then a stricter threshold
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
T=none,none,none,none,none,none,none,none
FLS_PLACEMENT_GOOD=0 timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 25 --rounds 3 --trials $T > $O/placement_q_sf25_r6q.txt 2>&1 || exit 1
FLS_PLACEMENT_GOOD=0 timeout -k 10 400 python3 -u scripts/placement_probe.py --workload c3 --scale 1 --rounds 3 --trials $T > $O/placement_q_c3_r6q.txt 2>&1 || exit 2
FLS_PLACEMENT_GOOD=990 FLS_PLACEMENT_TRIES=8 timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 25 --rounds 3 --trials none,none,none,none > $O/placement_g990_sf25_r6q.txt 2>&1 || exit 3
FLS_PLACEMENT_GOOD=990 FLS_PLACEMENT_TRIES=8 timeout -k 10 400 python3 -u scripts/placement_probe.py --workload c3 --scale 1 --rounds 3 --trials none,none,none,none > $O/placement_g990_c3_r6q.txt 2>&1 || exit 4
