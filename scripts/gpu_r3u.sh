# round 3u: narrowed delivery -- tests, then the e2e leg with and without it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_narrow.py tests/test_dict_codes.py tests/test_extension.py tests/test_filter.py tests/test_nulls.py tests/test_types.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_r3u.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r3u.log; grep -E "FAILED|Error" gpurun_out/pytest_r3u.log | head -20
[ $rc -ne 0 ] && exit $rc
for arm in narrow flat; do
  if [ $arm = flat ]; then export FLS_READ_NARROW=0; fi
  timeout -k 10 400 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-scale 10 --no-traffic > gpurun_out/bench_e2e_${arm}_r3u.json 2> gpurun_out/bench_e2e_${arm}_r3u.err
  rc=$?; echo "bench $arm rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_e2e_${arm}_r3u.json')); e=d.get('e2e'); print({k: e[k] for k in e if 'rows_s' in k})"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
