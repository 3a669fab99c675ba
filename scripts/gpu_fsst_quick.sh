#!/bin/bash
# FSST kernels: parity (FSST tests), then l_comment kernel times (SP vs CP)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_alp_fsst.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_fsstq.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_fsstq.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_fsstq.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/ab_env.py --workload lineitem_full --scale 10 --arms sp:FLS_DECODE_POLICY=0 cp:FLS_DECODE_POLICY=128 --cols 15 > gpurun_out/abenv_fsstq.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/abenv_fsstq.txt; exit $rc
