#!/bin/bash
# bench lines for BASELINE.json configs 3 and 4 (1e9-row INT64 delta keys,
# 1e9-row dictionary VARCHAR) next to the default SF100 line.
TAG=${1:-cfg}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c4; do
  timeout -k 10 600 python bench.py --workload $wl --steps 10 --cpu-seconds 5 > gpurun_out/bench_${wl}_$TAG.json 2> gpurun_out/bench_${wl}_$TAG.log
  rc=$?; echo "bench $wl rc=$rc"; cat gpurun_out/bench_${wl}_$TAG.json; [ $rc -eq 0 ] || exit $rc
done
