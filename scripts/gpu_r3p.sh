# round 3p: BOOLEAN / BLOB / CHAR and ROW_GROUPS_PER_FILE on the GPU
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_types.py tests/test_copy.py tests/test_writer.py tests/test_gpu_decode.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r3p.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r3p.log; exit $rc
