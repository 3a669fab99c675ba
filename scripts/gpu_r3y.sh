# round 3y: COPY A/B -- read_fastlanes with dictionary vectors (default) vs string_t (FLS_READ_DICT=0)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for arm in dict flat dict2; do
  if [ $arm = flat ]; then export FLS_READ_DICT=0; else unset FLS_READ_DICT; fi
  timeout -k 10 600 python scripts/writer_bench.py --scale 10 --threads 16 --copy --copy-only > gpurun_out/copy_${arm}_r3y.txt 2>&1
  rc=$?; echo "== $arm"; grep COPY gpurun_out/copy_${arm}_r3y.txt; [ $rc -eq 0 ] || exit $rc
done
