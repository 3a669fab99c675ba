# round 3v: e2e leg with / without narrowed delivery, extension built at -O3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for arm in narrow flat narrow2; do
  if [ $arm = flat ]; then export FLS_READ_NARROW=0; else unset FLS_READ_NARROW; fi
  timeout -k 10 400 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-scale 10 --no-traffic > gpurun_out/bench_e2e_${arm}_r3v.json 2> gpurun_out/bench_e2e_${arm}_r3v.err
  rc=$?; echo "bench $arm rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_e2e_${arm}_r3v.json')); e=d.get('e2e'); print({k: e[k] for k in e if 'rows_s' in k})"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
