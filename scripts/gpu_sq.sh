#!/bin/bash
# SQ issue/wait breakdown of the decode kernel per workload (one PMC pass each).
TAG=${1:-sq}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c4 lineitem; do
  timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU -d gpurun_out/sq_${wl}_$TAG -o pmc --output-format csv -- python3 bench.py --workload $wl --steps 2 --warmup 1 --cpu-seconds 0 --verify-rowgroups 0 --no-traffic > gpurun_out/sq_${wl}_$TAG.log 2>&1
  rc=$?; echo "sq $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
for wl in ("c3", "c4", "lineitem"):
    tot = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sq_{wl}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in tot.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 1)
    print(wl, {k: f"{v:.4g}" + (f" ({v / wc:.1%})" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else "") for k, v in sorted(avg.items())})
PY
