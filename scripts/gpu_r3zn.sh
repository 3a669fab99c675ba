# round 3zn: end-of-round check of the final tree (threshold 800): full GPU
# suite, smoke, default bench + rocprof, and the SF25 / SF12.5 shares
QUICK=1 bash scripts/gpu_round.sh r3zn || exit $?
cd $GRAFT_REPO_ROOT
for sf in 25 12.5; do
  timeout -k 10 400 python bench.py --scale $sf --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/bench_sf${sf}_r3zn.json 2> gpurun_out/bench_sf${sf}_r3zn.log
  rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/bench_sf${sf}_r3zn.json'));print('sf$sf', d['ms_per_step'], d['roofline']['frac'])"; [ $rc -eq 0 ] || exit $rc
done
