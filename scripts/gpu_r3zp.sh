# round 3zp: the final binary (with the W4 variant instantiated): full GPU
# suite and smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3/pytest_gpu_r3zp.log 2>&1
rc=$?; echo "pytest gpu rc=$rc: $(tail -1 gpurun_out/r3/pytest_gpu_r3zp.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke_r3zp.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/r3/smoke_r3zp.log)"; exit $rc
