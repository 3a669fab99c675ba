# copy kernel for the scan's D2H: GPU suite, then engine-scan A/B in fresh processes, then the bench
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_r6ao.log 2>&1 &&
timeout -k 10 500 python3 scripts/e2e_numa.py --runs 4 --brief --arms "kernel:FLS_SCAN_COPY_KERNEL=1;dma:FLS_SCAN_COPY_KERNEL=0" > $O/e2e_copy_ab_r6ao.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 5 --cpu-seconds 0 --no-traffic --no-verify > $O/bench_copyk_r6ao.json 2> $O/bench_copyk_r6ao.log
rc=$?
tail -2 $O/pytest_gpu_r6ao.log; cat $O/e2e_copy_ab_r6ao.txt
python3 -c "import json;d=json.load(open('$O/bench_copyk_r6ao.json'));e=d['e2e'];print('bench', round(d['ms_per_step'],3), 'engine', round(e['engine_scan_rows_s']/1e6), 'dc16', round(e['datachunk_rows_s_16t']/1e6), 'dc1', round(e['datachunk_rows_s_1t']/1e6), 'cold', round(e['datachunk_cold_rows_s_16t']/1e6))"
exit $rc
