# the whole GPU suite with the pinned arena on (every pinned buffer carved from never-released registered chunks), then the e2e block both ways
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
FLS_PIN_ARENA_MB=8192 timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu_arena_r6t.log 2>&1; rc=$?; echo "suite (arena) rc=$rc"; tail -1 $O/pytest_gpu_arena_r6t.log; [ $rc -eq 0 ] || exit $rc
for arm in 0 8192 0 8192; do
  FLS_PIN_ARENA_MB=$arm timeout -k 10 300 python3 bench.py --scale 1 --steps 2 --warmup 1 --cpu-seconds 0 --no-traffic --no-verify > $O/e2e_arena${arm}_r6t.json 2>/dev/null || exit 2
  python3 -c "import json;e=json.load(open('$O/e2e_arena${arm}_r6t.json'))['e2e'];print('arena=$arm cold', round(e['datachunk_cold_rows_s_16t']/1e6,1), 'warm16', round(e['datachunk_rows_s_16t']/1e6,1), 'warm1', round(e['datachunk_rows_s_1t']/1e6,1), 'engine', round(e['engine_scan_rows_s']/1e6,1))"
done
