# round 3q: NULL support on the GPU (C-ABI scan, filters, read_fastlanes / COPY round trips), then the filter/copy/extension suites
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nulls.py tests/test_filter.py tests/test_copy.py tests/test_extension.py tests/test_types.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r3q.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r3q.log; grep -E "FAILED|Error" gpurun_out/pytest_r3q.log | head -20; exit $rc
