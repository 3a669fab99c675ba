# round 3a: segmented FSST kernel parity + A/B, the 2-rank bench path
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3a.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "seg:FLS_FSST_SEG=1" "seg3072:FLS_FSST_SEG_CAP=3072" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_seg_r3a.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_launcher.py -m gpu > gpurun_out/r3/pt_launcher_r3a.log 2>&1 &&
timeout -k 10 500 python -u bench.py --gpus 2 --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/r3/bench_gpus2_sf100_r3a.json 2> gpurun_out/r3/bench_gpus2_sf100_r3a.err &&
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --e2e-scale 0 --no-traffic > gpurun_out/r3/bench_n1_r3a.json 2> gpurun_out/r3/bench_n1_r3a.err
