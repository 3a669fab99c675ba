# DELTA64 store order vs contiguous, c3 shape, same allocation per trial
mkdir -p gpurun_out; O=gpurun_out/membw11_r6au.txt
timeout -k 10 120 ./scripts/membw11 4 4 > $O 2>&1 && timeout -k 10 120 ./scripts/membw11 3 2 >> $O 2>&1
rc=$?; cat $O; exit $rc
