#!/bin/bash
# SQ counters of one FSST kernel on l_comment (lineitem_full SF10).
# usage: gpu_fsst_sq.sh [kernel-name-substring] [tag]   (default fsst_sp_kernel)
K=${1:-fsst_sp_kernel}
TAG=${2:-sp}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAVES"
P3="SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/fsq_${TAG}$i -o pmc --output-format csv -- python3 scripts/fsst_prof.py > gpurun_out/fsq_${TAG}$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/fsq_${TAG}$i.log; exit $rc; }
done
K=$K TAG=$TAG python3 - <<'PY'
import csv, glob, collections, os
tot = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/fsq_{os.environ['TAG']}*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if os.environ["K"] in r["Kernel_Name"]:
            tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in tot.items()}
wc = avg.get("SQ_WAVE_CYCLES", 1)
for k, v in sorted(avg.items()):
    print(f"{k:24s} {v:14.4g}" + (f"  ({v / wc:.1%} of wave cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""))
PY
