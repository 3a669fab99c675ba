#!/bin/bash
# Default bench (the driver's command) + a kernel-trace profile of the same run.
# usage: bash scripts/gpu_bench_r2.sh <tag> [extra bench args]
TAG=${1:-r2}
shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.log
exit $rc
