# placement search A/B at bench level (separate processes, interleaved), then the touched GPU tests
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 120 ./scripts/pin_probe 8 200 > $O/pin_probe_r6k.txt 2>&1; echo "pin_probe rc=$?"; cat $O/pin_probe_r6k.txt
B="python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic --no-verify"
for i in 1 2 3; do
  for arm in 1 4; do
    FLS_PLACEMENT_TRIES=$arm timeout -k 10 200 $B --scale 12.5 > $O/abpl_sf12_t${arm}_$i.json 2> $O/abpl_sf12_t${arm}_$i.log || exit 1
    python3 -c "import json;d=json.load(open('$O/abpl_sf12_t${arm}_$i.json'));print('sf12.5 tries=$arm run $i', d['ms_per_step'], d['roofline']['frac'])"
  done
done
for i in 1 2; do
  for arm in 1 4; do
    FLS_PLACEMENT_TRIES=$arm timeout -k 10 300 $B --scale 100 > $O/abpl_sf100_t${arm}_$i.json 2> $O/abpl_sf100_t${arm}_$i.log || exit 2
    python3 -c "import json;d=json.load(open('$O/abpl_sf100_t${arm}_$i.json'));print('sf100 tries=$arm run $i', d['ms_per_step'], d['roofline']['frac'])"
  done
done
for i in 1 2; do
  for arm in 1 4; do
    FLS_PLACEMENT_TRIES=$arm timeout -k 10 200 $B --workload c3 > $O/abpl_c3_t${arm}_$i.json 2> $O/abpl_c3_t${arm}_$i.log || exit 3
    python3 -c "import json;d=json.load(open('$O/abpl_c3_t${arm}_$i.json'));print('c3 tries=$arm run $i', d['ms_per_step'], d['roofline']['frac'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_alp_fsst.py tests/test_gpu_multi.py tests/test_resident_scan.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r6k.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest_r6k.log
