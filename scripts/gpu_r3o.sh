# round 3o: GPU tests touched by the pinned-memory cap, COPY staging and the FSST LDS check
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_open_cache.py tests/test_copy.py tests/test_alp_fsst.py tests/test_extension.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r3o.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r3o.log; exit $rc
