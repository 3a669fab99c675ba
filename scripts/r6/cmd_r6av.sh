# the copy-kernel D2H with the opt-in registered arena: scan suites, then cold queries both ways
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
FLS_PIN_ARENA_MB=8192 timeout -k 10 500 python -u -m pytest tests/test_scan_copy.py tests/test_resident_scan.py tests/test_narrow.py tests/test_filter.py tests/test_extension.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_scan_arena_r6av.log 2>&1 &&
timeout -k 10 600 python3 scripts/cold_query.py --runs 3 --warm 3 --arms "hm:FLS_PIN_ARENA_MB=0;arena:FLS_PIN_ARENA_MB=8192" > $O/cold_arena_r6av.txt 2>&1
rc=$?
tail -2 $O/pytest_scan_arena_r6av.log; cat $O/cold_arena_r6av.txt
exit $rc
