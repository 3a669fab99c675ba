#!/bin/bash
# Round checkpoint: GPU tests, smoke, default bench (with PMC traffic), rocprof
# kernel stats of the default bench, config 3/4 and ALP/FSST bench lines,
# per-column rates.  usage: gpu_round.sh <tag>
TAG=${1:-r}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest gpu rc=$rc: $(tail -1 gpurun_out/pytest_gpu_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/smoke_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec head -3 {} \; ; [ $rc -eq 0 ] || exit $rc
[ -n "$QUICK" ] && exit 0
for wl in c3 c4 lineitem_full lineitem_dbl; do
  timeout -k 10 500 python bench.py --workload $wl --steps 10 --cpu-seconds 5 > gpurun_out/bench_${wl}_$TAG.json 2> gpurun_out/bench_${wl}_$TAG.log
  rc=$?; echo "bench $wl rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench_${wl}_$TAG.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['frac'],d['roofline']['traffic'])"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/percol.py --workload lineitem_full --scale 10 > gpurun_out/percol_$TAG.txt 2>&1
rc=$?; echo "percol rc=$rc"; grep -v amdgpu gpurun_out/percol_$TAG.txt; exit $rc
