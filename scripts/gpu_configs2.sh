#!/bin/bash
# Bench lines for the non-headline configurations plus per-column rates.
# usage: gpu_configs2.sh <tag>
TAG=${1:-r}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c4 lineitem_full lineitem_dbl; do
  timeout -k 10 500 python bench.py --workload $wl --steps 10 --cpu-seconds 5 > gpurun_out/bench_${wl}_$TAG.json 2> gpurun_out/bench_${wl}_$TAG.log
  rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${wl}_$TAG.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['frac'],d['roofline']['traffic'])"
done
timeout -k 10 300 python scripts/percol.py --workload lineitem_full --scale 10 > gpurun_out/percol_$TAG.txt 2>&1
rc=$?; echo "percol rc=$rc"; grep -v amdgpu gpurun_out/percol_$TAG.txt; exit $rc
