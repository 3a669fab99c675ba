#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d gpurun_out/fsq$i -o pmc --output-format csv -- python3 scripts/fsst_prof.py > gpurun_out/fsq$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(list)
for f in glob.glob("gpurun_out/fsq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fsst_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in tot.items()}
wc = avg.get("SQ_WAVE_CYCLES", 1)
for k, v in sorted(avg.items()):
    print(f"{k:24s} {v:14.4g}" + (f"  ({v / wc:.1%} of wave cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""))
PY
