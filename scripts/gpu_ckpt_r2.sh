#!/bin/bash
# Round-2 checkpoint: GPU tests + smoke, the default bench, a kernel-trace
# profile of the bench command, and the per-GPU share of an 8-GPU run
# (SF100 / 8 = SF12.5 on one GPU) as a scaling rehearsal.
TAG=${1:-r2e}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r2.sh $TAG || exit $?
bash scripts/gpu_bench_r2.sh $TAG || exit $?
timeout -k 10 400 python -u bench.py --scale 12.5 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/bench_sf12p5_$TAG.json 2> gpurun_out/bench_sf12p5_$TAG.log
rc=$?; echo "sf12.5 rc=$rc"; cat gpurun_out/bench_sf12p5_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.log
rc=$?; echo "prof rc=$rc"; find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$TAG.csv \; ; head -5 gpurun_out/kernel_stats_$TAG.csv
exit $rc
