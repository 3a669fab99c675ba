cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showmeminfo vram > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/host.txt; lscpu | head -20 >> gpurun_out/host.txt; free -g >> gpurun_out/host.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --scale 1 --steps 10 --cpu-seconds 3 > gpurun_out/bench_sf1.json 2> gpurun_out/bench_sf1.log
rc=$?; echo "bench sf1 rc=$rc"; cat gpurun_out/bench_sf1.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --cpu-seconds 5 > gpurun_out/bench_sf100.json 2> gpurun_out/bench_sf100.log
rc=$?; echo "bench sf100 rc=$rc"; cat gpurun_out/bench_sf100.json; exit $rc
