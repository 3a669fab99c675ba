# scan slots in flight with the copy-kernel D2H: warm 16-thread DataChunk queries, interleaved fresh processes
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 900 python3 scripts/cold_query.py --runs 4 --warm 5 --arms "s2:FLS_SCAN_SLOTS=2;s3:FLS_SCAN_SLOTS=3" > $O/slots_r6az.txt 2>&1
rc=$?; cat $O/slots_r6az.txt; exit $rc
