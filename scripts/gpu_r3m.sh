# round 3m: full GPU suite, smoke, default bench + rocprof (QUICK round), then the 8-GPU share (SF12.5)
QUICK=1 bash scripts/gpu_round.sh r3m || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --scale 12.5 --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/bench_sf12p5_r3m.json 2> gpurun_out/bench_sf12p5_r3m.log
rc=$?; echo "bench sf12.5 rc=$rc"; cat gpurun_out/bench_sf12p5_r3m.json | head -c 400; exit $rc
