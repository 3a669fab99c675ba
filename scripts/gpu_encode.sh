#!/bin/bash
# GPU encoder: parity tests, device-resident rates, writer rates, rocprof stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encode.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_encode.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_encode.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_encode.log | head -30; tail -30 gpurun_out/pt_encode.log; exit $rc; }
timeout -k 10 600 python scripts/encode_bench.py > gpurun_out/encode_bench.txt 2>&1
rc=$?; echo "== bench rc=$rc"; grep -v amdgpu gpurun_out/encode_bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o kt --output-format csv -- python3 scripts/encode_bench.py --no-writer --reps 3 > gpurun_out/prof_enc.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_enc -name "*kernel_stats.csv" -exec cat {} \; ; exit $rc
