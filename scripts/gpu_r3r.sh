# round 3r: dictionary-coded delivery (engine + read_fastlanes), extension suites, then the e2e bench leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dict_codes.py tests/test_extension.py tests/test_filter.py tests/test_nulls.py tests/test_copy.py tests/test_types.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_r3r.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r3r.log; grep -E "FAILED|Error" gpurun_out/pytest_r3r.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-scale 10 --no-traffic > gpurun_out/bench_e2e_r3r.json 2> gpurun_out/bench_e2e_r3r.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_e2e_r3r.json')); print(json.dumps(d.get('e2e'), indent=1))"
[ $rc -ne 0 ] && exit $rc
FLS_READ_DICT=0 timeout -k 10 400 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-scale 10 --no-traffic > gpurun_out/bench_e2e_flat_r3r.json 2> gpurun_out/bench_e2e_flat_r3r.err
rc=$?; echo "bench flat rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_e2e_flat_r3r.json')); print(json.dumps(d.get('e2e'), indent=1))"
exit $rc
