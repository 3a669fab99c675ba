# third slot on recycled host batches only: scan suites with 3 slots, then 2 vs 3 slots (cold + warm), fresh processes
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
FLS_SCAN_SLOTS=3 timeout -k 10 600 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py tests/test_narrow.py tests/test_filter.py tests/test_extension.py tests/test_scan_errors.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_scan_s3_r6ba.log 2>&1 &&
timeout -k 10 900 python3 scripts/cold_query.py --runs 4 --warm 5 --arms "s2:FLS_SCAN_SLOTS=2;s3:FLS_SCAN_SLOTS=3" > $O/slots_lazy_r6ba.txt 2>&1
rc=$?; tail -2 $O/pytest_scan_s3_r6ba.log; cat $O/slots_lazy_r6ba.txt; exit $rc
