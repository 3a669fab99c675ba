#!/bin/bash
# GPU validation round: build, GPU parity tests, smoke, default bench.
# usage: bash scripts/gpu_test.sh <tag>
TAG=${1:-t}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/smoke_$TAG.log
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc3=$?; echo "bench rc=$rc3"; cat gpurun_out/bench_$TAG.json
[ $rc3 -eq 0 ] || exit $rc3
# same bench without the PMC child passes (checks they do not perturb timing)
timeout -k 10 400 python bench.py --no-traffic --cpu-seconds 0 > gpurun_out/bench_${TAG}_nt.json 2>> gpurun_out/bench_$TAG.log
rc4=$?; echo "bench(no traffic) rc=$rc4"; cat gpurun_out/bench_${TAG}_nt.json
exit $((rc + rc4))
