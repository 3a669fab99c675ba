#!/bin/bash
# scan-pipeline batches: decode kernel time under the default policy (small
# launches -> balanced split) vs the forced work queue (64); e2e rates of both.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_extension.py tests/test_filter.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_scanpol.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_scanpol.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pt_scanpol.log; exit $rc; }
for p in 0 64; do
  FLS_DECODE_POLICY=$p timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_scan_p$p -o kt --output-format csv -- python3 scripts/e2e.py --scale 10 > gpurun_out/e2e_scan_p$p.txt 2>&1
  rc=$?; echo "== policy $p rc=$rc"; grep -v amdgpu.ids gpurun_out/e2e_scan_p$p.txt | head -8; find gpurun_out/prof_scan_p$p -name "*kernel_stats.csv" -exec cat {} \; ; [ $rc -eq 0 ] || exit $rc
done
