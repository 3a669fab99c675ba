# blocking vs polling wait for a batch's event: warm/cold 16-thread queries, interleaved fresh processes
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 900 python3 scripts/cold_query.py --runs 4 --warm 5 --arms "block:FLS_SCAN_SPIN_WAIT=0;spin:FLS_SCAN_SPIN_WAIT=1" > $O/spin_wait_r6be.txt 2>&1
rc=$?; cat $O/spin_wait_r6be.txt; exit $rc
