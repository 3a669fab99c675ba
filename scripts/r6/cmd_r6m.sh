# non-temporal output stores vs plain: SF100 headline, c4, lineitem (15 cols) SF10; placement re-drawn every round
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 900 python -u scripts/ab_builds.py --variants base,nts --workload lineitem_full --scale 100 --rounds 4 --reps 3 > $O/ab_builds_nt_sf100_r6m.txt 2>&1; echo "sf100 rc=$?"; tail -1 $O/ab_builds_nt_sf100_r6m.txt
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,nts --workload c4 --scale 1 --rounds 6 --verify > $O/ab_builds_nt_c4_r6m.txt 2>&1; echo "c4 rc=$?"; tail -1 $O/ab_builds_nt_c4_r6m.txt
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,nts --workload lineitem --scale 10 --rounds 6 --verify > $O/ab_builds_nt_li10_r6m.txt 2>&1; echo "li rc=$?"; tail -1 $O/ab_builds_nt_li10_r6m.txt
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,nts --workload c3 --scale 1 --rounds 6 --verify > $O/ab_builds_nt_c3_r6m.txt 2>&1; echo "c3 rc=$?"; tail -1 $O/ab_builds_nt_c3_r6m.txt
