#!/bin/bash
# Measurement of the widened rows: ALP / FSST bench lines,
# per-column rates of lineitem_full, writer + COPY rates; full GPU test suite first.
TAG=${1:-w}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C duckdb-fastlane_amd && make -s -C oracle || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest gpu rc=$rc: $(tail -1 gpurun_out/pytest_gpu_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
for wl in lineitem_full lineitem_dbl; do
  timeout -k 10 600 python bench.py --workload $wl --steps 10 --cpu-seconds 5 > gpurun_out/bench_${wl}_$TAG.json 2> gpurun_out/bench_${wl}_$TAG.log
  rc=$?; echo "bench $wl rc=$rc"; cat gpurun_out/bench_${wl}_$TAG.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/percol.py --workload lineitem_full --scale 10 > gpurun_out/percol_full_$TAG.txt 2>&1
rc=$?; echo "percol rc=$rc"; grep -v amdgpu gpurun_out/percol_full_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/writer_bench.py --scale 10 --threads 16 --copy > gpurun_out/writer_$TAG.txt 2>&1
rc=$?; echo "writer rc=$rc"; grep -v amdgpu gpurun_out/writer_$TAG.txt; exit $rc
