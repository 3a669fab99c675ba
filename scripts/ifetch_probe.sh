#!/bin/bash
# Instruction-fetch counters of interleaved decode launches from two builds
# loaded in one process (scripts/ab.py): which counters differ between the
# first- and second-loaded build.  Usage: scripts/ifetch_probe.sh <tag> <variants> <scale>
TAG=$1; VARS=$2; SC=${3:-12.5}
O=gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > $O/counters_$TAG.txt 2>&1
grep -i -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INSTS_[A-Z_]*" $O/counters_$TAG.txt | sort -u | head -40
P="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES"
timeout -k 10 -s KILL 240 rocprofv3 --pmc $P -d $O/ifq_${TAG}_1 -o pmc --output-format csv -- \
    python3 scripts/ab.py --variants "$VARS" --workload lineitem_full --scale "$SC" --cols all --rounds 2 --reps 1 \
    > $O/ifq_${TAG}_1.log 2>&1
rc=$?; echo "pmc pass 1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/ifq_${TAG}_1.log; exit $rc; }
P2="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ"
timeout -k 10 -s KILL 240 rocprofv3 --pmc $P2 -d $O/ifq_${TAG}_2 -o pmc --output-format csv -- \
    python3 scripts/ab.py --variants "$VARS" --workload lineitem_full --scale "$SC" --cols all --rounds 2 --reps 1 \
    > $O/ifq_${TAG}_2.log 2>&1
rc=$?; echo "pmc pass 2 rc=$rc"; [ $rc -eq 0 ] || tail -5 $O/ifq_${TAG}_2.log
exit 0
