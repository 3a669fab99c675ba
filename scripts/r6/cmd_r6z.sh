# decode-time rating vs write-probe rating at SF12.5 (ratings and the kept set's measured decode)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 12.5 --rounds 4 --trials none,none,none,none,none,none > $O/placement_dec_sf12_r6z.txt 2>&1 || exit 1
FLS_PLACEMENT_DECODE=0 timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 12.5 --rounds 4 --trials none,none,none,none,none,none > $O/placement_probe_sf12_r6z.txt 2>&1 || exit 2
FLS_PLACEMENT_DECODE=8 timeout -k 10 400 python3 -u scripts/placement_probe.py --scale 12.5 --rounds 4 --trials none,none,none,none > $O/placement_dec8_sf12_r6z.txt 2>&1 || exit 3
