export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 400 python3 -u scripts/placement_probe.py --rounds 5 --trials none,bestof:4,none,bestof:4,none,bestof:4,none,bestof:4 > $O/placement_bestof_r6f.txt 2>&1 || exit 2
timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 100 --rounds 3 --trials none,bestof:3,none,bestof:3 > $O/placement_bestof_sf100_r6f.txt 2>&1 || exit 3
