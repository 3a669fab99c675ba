# round 3w: narrowed read_fastlanes tests, then the default e2e leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_narrow.py tests/test_dict_codes.py tests/test_extension.py tests/test_filter.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_r3w.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r3w.log; grep -E "FAILED|Error" gpurun_out/pytest_r3w.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-scale 10 --no-traffic > gpurun_out/bench_e2e_r3w.json 2> gpurun_out/bench_e2e_r3w.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_e2e_r3w.json')); e=d.get('e2e'); print({k: e[k] for k in e if 'rows_s' in k})"
exit $rc
