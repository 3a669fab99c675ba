set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_launcher.py -m gpu > gpurun_out/r3/pt_launcher.log 2>&1 &&
timeout -k 10 500 python -u bench.py --gpus 2 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/r3/bench_gpus2_sf100.json 2> gpurun_out/r3/bench_gpus2_sf100.err &&
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/r3/bench_n1_sf100.json 2> gpurun_out/r3/bench_n1_sf100.err
