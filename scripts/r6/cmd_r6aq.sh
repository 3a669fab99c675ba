# copy kernel H2D too: new parity test + scan suites, cold-query A/B in fresh processes
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_scan_r6aq.log 2>&1 &&
timeout -k 10 600 python3 scripts/cold_query.py --runs 3 --warm 3 --arms "kernel:FLS_SCAN_COPY_KERNEL=1;dma:FLS_SCAN_COPY_KERNEL=0" > $O/cold_copy_ab_r6aq.txt 2>&1
rc=$?
tail -2 $O/pytest_scan_r6aq.log; cat $O/cold_copy_ab_r6aq.txt
exit $rc
