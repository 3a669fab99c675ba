# cached occupancy queries: decode/FSST/scan tests, then the refill profile again
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_alp_fsst.py tests/test_gpu_decode.py tests/test_scan_copy.py tests/test_extension.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_occ_r6bd.log 2>&1 &&
timeout -k 10 300 python3 scripts/cold_query.py --runs 1 --warm 3 --profile > $O/refill_prof_r6bd.txt 2>&1 &&
timeout -k 10 600 python3 scripts/cold_query.py --runs 3 --warm 5 > $O/cold_occ_r6bd.txt 2>&1
rc=$?; tail -2 $O/pytest_occ_r6bd.log; grep -E "fill|seen|cold|warm" $O/refill_prof_r6bd.txt | tail -8; cat $O/cold_occ_r6bd.txt; exit $rc
