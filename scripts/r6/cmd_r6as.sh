# host columns at the delivered width: scan suites, then cold queries in fresh processes (profiled)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py tests/test_narrow.py tests/test_filter.py tests/test_extension.py tests/test_nulls.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_scan_r6as.log 2>&1 &&
timeout -k 10 600 python3 scripts/cold_query.py --runs 3 --warm 3 > $O/cold_width_r6as.txt 2>&1 &&
timeout -k 10 300 python3 scripts/cold_query.py --runs 1 --warm 1 --profile > $O/cold_width_prof_r6as.txt 2>&1
rc=$?
tail -2 $O/pytest_scan_r6as.log; cat $O/cold_width_r6as.txt
exit $rc
