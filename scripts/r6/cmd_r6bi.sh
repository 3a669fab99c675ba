# memoized chunk metadata sums in the scan's refill: scan suites, profile, warm A/B
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py tests/test_narrow.py tests/test_filter.py tests/test_extension.py tests/test_alp_fsst.py tests/test_gpu_decode.py tests/test_nulls.py tests/test_scan_errors.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_cstat_r6bi.log 2>&1 &&
timeout -k 10 300 python3 scripts/cold_query.py --runs 1 --warm 3 --profile > $O/refill_prof_r6bi.txt 2>&1 &&
timeout -k 10 900 python3 scripts/cold_query.py --runs 3 --warm 5 --arms "stat:FLS_SCAN_NO_CHUNKSTAT=0;walk:FLS_SCAN_NO_CHUNKSTAT=1" > $O/cstat_ab_r6bi.txt 2>&1
rc=$?; tail -2 $O/pytest_cstat_r6bi.log; grep -E "fill|seen" $O/refill_prof_r6bi.txt | tail -4; cat $O/cstat_ab_r6bi.txt; exit $rc
