#!/bin/bash
# Profile round: per-column roofline, bench, rocprofv3 kernel trace + PMC passes.
# usage: bash scripts/gpu_prof.sh <tag>
TAG=${1:-r1}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 300 python scripts/percol.py --scale 10 > gpurun_out/percol_$TAG.txt 2>&1
rc=$?; echo "percol rc=$rc"; cat gpurun_out/percol_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python3 bench.py --steps 10 --cpu-seconds 0 --verify-rowgroups 0 --no-traffic > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --verify-rowgroups 0 --no-traffic > gpurun_out/pmc_fetch_$TAG.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --verify-rowgroups 0 --no-traffic > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; exit $rc
