export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 200 ./scripts/membw7 12 > $O/membw7_r6d.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/placement_probe.py --rounds 5 --trials none,none,none,none,none,none,none,none,none,none,none,none > $O/placement_many_r6d.txt 2>&1 || exit 2
