# round 3zj: FSST columns delivered as string lengths (records rebuilt on the
# consumer's thread) -- narrow / dictionary / extension GPU tests, then the
# e2e rates of lineitem_full SF10 (bench e2e leg only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_narrow.py tests/test_dict_codes.py tests/test_extension.py tests/test_nulls.py -m gpu > gpurun_out/r3/pt_strlen_r3zj.log 2>&1
rc=$?; tail -3 gpurun_out/r3/pt_strlen_r3zj.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --scale 1 --steps 3 --warmup 1 --cpu-seconds 0 --no-traffic --e2e-scale 10 > gpurun_out/r3/bench_e2e_strlen_r3zj.json 2> gpurun_out/r3/bench_e2e_strlen_r3zj.log
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/r3/bench_e2e_strlen_r3zj.json'));print(json.dumps(d['e2e']))"; exit $rc
