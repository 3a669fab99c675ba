#!/bin/bash
# Round-2 GPU validation: host facts, GPU parity tests (one process), smoke.
# usage: bash scripts/gpu_r2.sh <tag> [pytest -k expr]
TAG=${1:-r2}
K=${2:-}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
(nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max;
 lscpu | head -30; free -g) > gpurun_out/hostinfo_$TAG.txt 2>&1
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA "${KARG[@]}" --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -25 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/smoke_$TAG.log
exit $((rc + rc2))
