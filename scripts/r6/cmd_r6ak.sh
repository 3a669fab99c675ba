# engine-scan bimodality: NUMA node of pinned buffers, fresh processes, before and after a bench run
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
cat /sys/devices/system/node/online > $O/numa_r6ak.txt 2>&1 || true
timeout -k 10 300 python3 scripts/e2e_numa.py --runs 2 > $O/e2e_numa_r6ak.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 5 --cpu-seconds 0 --no-traffic --no-verify > $O/e2e_numa_bench_r6ak.json 2> $O/e2e_numa_bench_r6ak.log &&
timeout -k 10 300 python3 scripts/e2e_numa.py --runs 2 >> $O/e2e_numa_r6ak.txt 2>&1
rc=$?
cat $O/numa_r6ak.txt $O/e2e_numa_r6ak.txt
python3 -c "import json;d=json.load(open('$O/e2e_numa_bench_r6ak.json'));e=d['e2e'];print('bench', round(d['ms_per_step'],3), 'engine', round(e['engine_scan_rows_s']/1e6), 'dc16', round(e['datachunk_rows_s_16t']/1e6))"
exit $rc
