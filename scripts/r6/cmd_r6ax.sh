# early slot refill: scan/extension suites, then warm+cold A/B in fresh processes
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py tests/test_narrow.py tests/test_filter.py tests/test_extension.py tests/test_scan_errors.py tests/test_nulls.py tests/test_gpu_multi.py tests/test_resident_budget.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_scan_r6ax.log 2>&1 &&
timeout -k 10 900 python3 scripts/cold_query.py --runs 3 --warm 5 --arms "early:FLS_SCAN_EARLY_REFILL=1;late:FLS_SCAN_EARLY_REFILL=0" > $O/early_refill_r6ax.txt 2>&1 &&
timeout -k 10 500 python3 scripts/e2e_numa.py --runs 2 --brief --arms "early:FLS_SCAN_EARLY_REFILL=1;late:FLS_SCAN_EARLY_REFILL=0" > $O/early_refill_engine_r6ax.txt 2>&1
rc=$?
tail -2 $O/pytest_scan_r6ax.log; cat $O/early_refill_r6ax.txt $O/early_refill_engine_r6ax.txt
exit $rc
