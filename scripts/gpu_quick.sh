#!/bin/bash
# Quick GPU check: build, then the GPU test suite (optionally a -k filter).
TAG=${1:-q}
K=${2:-}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -rA -p no:cacheprovider -k "$K" > gpurun_out/pytest_gpu_$TAG.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
fi
rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | tail -15
exit $rc
