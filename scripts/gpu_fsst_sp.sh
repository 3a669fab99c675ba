#!/bin/bash
# string-parallel FSST: full GPU parity, then same-buffer A/B against the
# code-parallel kernel (policy 128) on l_comment, and the lineitem_full bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_fsst_sp.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_fsst_sp.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_fsst_sp.log | head -30; tail -40 gpurun_out/pt_fsst_sp.log; exit $rc; }
timeout -k 10 600 python scripts/ab_env.py --workload lineitem_full --scale 10 --arms sp:FLS_DECODE_POLICY=0 cp:FLS_DECODE_POLICY=128 --cols all,15 > gpurun_out/abenv_fsst_sp.txt 2>&1
rc=$?; echo "== ab"; grep -v amdgpu gpurun_out/abenv_fsst_sp.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --workload lineitem_full --steps 10 --cpu-seconds 5 > gpurun_out/bench_lineitem_full_sp.json 2> gpurun_out/bench_lineitem_full_sp.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_lineitem_full_sp.json; exit $rc
