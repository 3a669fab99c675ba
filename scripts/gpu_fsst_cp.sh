#!/bin/bash
# code-parallel FSST (parity-rule escapes, qword writer, deferred stores):
# GPU parity (all GPU tests, or FSST only with QUICK=1), a same-buffer A/B
# against the string-parallel kernel on l_comment, then the lineitem_full bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=tests; [ -n "$QUICK" ] && T=tests/test_alp_fsst.py
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_fsst_cp.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_fsst_cp.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_fsst_cp.log | head -30; tail -40 gpurun_out/pt_fsst_cp.log; exit $rc; }
timeout -k 10 600 python scripts/ab_env.py --workload lineitem_full --scale 10 --arms sp:FLS_DECODE_POLICY=128 cp8:FLS_DECODE_POLICY=0 --cols 15 > gpurun_out/abenv_fsst_cp.txt 2>&1
rc=$?; echo "== ab"; grep -v amdgpu gpurun_out/abenv_fsst_cp.txt; [ $rc -eq 0 ] || exit $rc
[ -n "$QUICK" ] && exit 0
timeout -k 10 500 python bench.py --workload lineitem_full --steps 10 --cpu-seconds 5 > gpurun_out/bench_lineitem_full_cp.json 2> gpurun_out/bench_lineitem_full_cp.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_lineitem_full_cp.json; exit $rc
