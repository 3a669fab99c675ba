#!/bin/bash
# Bench lines for the other BASELINE.json configs on the current build:
# c1 (1e6 INT32), c3 (1e9 INT64 DELTA keys), c4 (1e9 dictionary VARCHAR),
# lineitem (15 columns) and lineitem_dbl (ALP doubles) at SF100.
TAG=${1:-r2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c1 c3 c4 lineitem lineitem_dbl; do
  timeout -k 10 600 python bench.py --workload $wl --steps 10 --cpu-seconds 4 --e2e-scale 0 > gpurun_out/bench_${wl}_$TAG.json 2> gpurun_out/bench_${wl}_$TAG.log
  rc=$?; echo "bench $wl rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['metric'], '%.3e'%d['value'], 'kernel %.3f ms'%r['kernel_ms'], 'frac %.3f'%r['frac'], 'traffic', r['traffic'], 'algo %.3f GB'%(r['algo_bytes_per_launch']/1e9), 'cpu %.3e'%d['cpu_baseline']['value'], 'verified', d['config']['verified_values_bit_exact'])" gpurun_out/bench_${wl}_$TAG.json; [ $rc -eq 0 ] || exit $rc
done
