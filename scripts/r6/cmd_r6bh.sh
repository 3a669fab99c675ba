# where a warm query's refill latency goes (FLS_SCAN_PROFILE sub-phases)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python3 scripts/cold_query.py --runs 1 --warm 3 --profile > $O/refill_prof_r6bh.txt 2>&1
rc=$?; grep -v "^\s*$" $O/refill_prof_r6bh.txt | head -80; exit $rc
