# round 3zk: final checkpoint of round 3 -- full GPU suite, smoke, default
# bench (PMC traffic) + rocprof kernel stats, and the 8-GPU per-GPU share
# (SF12.5) on one GPU
QUICK=1 bash scripts/gpu_round.sh r3zk || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --scale 12.5 --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/bench_sf12p5_r3zk.json 2> gpurun_out/bench_sf12p5_r3zk.log
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/bench_sf12p5_r3zk.json'));print('sf12.5', d['ms_per_step'], d['roofline']['frac'])"; exit $rc
