#!/bin/bash
# Filter pushdown measurement: e2e rates (with / without WHERE) and a
# rocprofv3 kernel trace of the same run (decode / filter / compact kernels).
TAG=${1:-f}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 600 python scripts/e2e.py --scale 10 > gpurun_out/e2e_$TAG.txt 2>&1
rc=$?; echo "e2e rc=$rc"; grep -v amdgpu.ids gpurun_out/e2e_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e_$TAG -o kt --output-format csv -- python3 scripts/e2e.py --scale 10 > gpurun_out/prof_e2e_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_e2e_$TAG -name "*kernel_stats.csv" -exec cat {} \; ; exit $rc
