#!/bin/bash
# Per-GPU share of an 8-GPU run (SF100 / 8 = SF12.5) on one GPU: kernel
# traces of the 16-column step overlapped (default) and serial
# (FLS_OVERLAP_FSST_WPC=0), and the 15-column step without FSST, to locate
# where the small share loses rate against SF100.
TAG=${1:-sf12}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--scale ${SCALE:-12.5} --steps 10 --warmup 2 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic"
for arm in ${ARMS:-ovl ser l15}; do
  case $arm in
    ovl) W=lineitem_full; export FLS_OVERLAP_FSST_WPC=12 ;;
    ser) W=lineitem_full; export FLS_OVERLAP_FSST_WPC=0 ;;
    l15) W=lineitem; unset FLS_OVERLAP_FSST_WPC ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_${TAG}_$arm -o tr -- python3 bench.py --workload $W $B \
    > gpurun_out/tr_${TAG}_$arm.json 2> gpurun_out/tr_${TAG}_$arm.log
  rc=$?; echo "$arm rc=$rc"; cat gpurun_out/tr_${TAG}_$arm.json; [ $rc -eq 0 ] || exit $rc
  db=$(find gpurun_out/tr_${TAG}_$arm -name "*.db" | head -1)
  /opt/rocm/bin/rocpd2csv -i $db -d gpurun_out/tr_${TAG}_$arm > /dev/null 2>&1
  rm -f $db
done
exit 0
