#!/bin/bash
# Default bench (as the driver runs it) + end-to-end DataChunk delivery rate.
TAG=${1:-b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; grep -v amdgpu.ids gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/e2e.py > gpurun_out/e2e_$TAG.txt 2>&1
rc=$?; echo "e2e rc=$rc"; grep -v amdgpu.ids gpurun_out/e2e_$TAG.txt; exit $rc
