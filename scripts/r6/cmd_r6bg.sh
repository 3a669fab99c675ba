# the scan batch's decode grid (latency-bound, 264 us per batch): warm 16-thread queries by env arm
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 1000 python3 scripts/cold_query.py --runs 3 --warm 5 --arms "def:;bpc1:FLS_BLOCKS_PER_CU=1;bpc2:FLS_BLOCKS_PER_CU=2;tp1:FLS_TAIL_PIECES=1" > $O/scan_grid_r6bg.txt 2>&1
rc=$?; cat $O/scan_grid_r6bg.txt; exit $rc
