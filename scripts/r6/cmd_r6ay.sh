# kernel timeline of warm 16-thread read_fastlanes queries: does the D2H copy kernel keep the link busy?
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python3 scripts/cold_query.py --gen-only /tmp/li10.fls > $O/tl_gen_r6ay.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_r6ay -o kt --output-format csv -- python3 scripts/cold_query.py --child /tmp/li10.fls --threads 16 --warm 4 > $O/tl_run_r6ay.log 2>&1 &&
python3 scripts/scan_timeline.py $(find $O/tl_r6ay -name "*kernel_trace.csv" | head -1) > $O/scan_timeline_r6ay.txt 2>&1
rc=$?; tail -1 $O/tl_run_r6ay.log; cat $O/scan_timeline_r6ay.txt; exit $rc
