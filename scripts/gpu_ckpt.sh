#!/bin/bash
# Checkpoint: all GPU tests, smoke, default bench (PMC traffic, CPU baseline),
# rocprof kernel stats of it, lineitem_full bench.  usage: gpu_ckpt.sh <tag>
TAG=${1:-r}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest gpu rc=$rc: $(tail -1 gpurun_out/pytest_gpu_$TAG.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu_$TAG.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/smoke_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python3 bench.py --steps 20 --cpu-seconds 0 --verify-rowgroups 0 --no-traffic > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec head -3 {} \; ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --workload lineitem_full --steps 10 --cpu-seconds 5 > gpurun_out/bench_lineitem_full_$TAG.json 2> gpurun_out/bench_lineitem_full_$TAG.log
rc=$?; echo "bench lineitem_full rc=$rc"; cat gpurun_out/bench_lineitem_full_$TAG.json; exit $rc
