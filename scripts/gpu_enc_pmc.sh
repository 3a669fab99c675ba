#!/bin/bash
# HBM traffic of the encoder kernels: one rocprofv3 --pmc pass per counter over
# the device-resident encode cases (each case: warm-up + 1 timed launch).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_enc_$ctr -o pmc --output-format csv -- python3 scripts/encode_bench.py --no-writer --reps 1 > gpurun_out/pmc_enc_$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
