# pin probe with forced address reuse; the 8-way split tests; cold-query arena A/B
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 120 ./scripts/pin_probe 8 200 > $O/pin_probe_r6l.txt 2>&1; echo "pin_probe rc=$?"; cat $O/pin_probe_r6l.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_resident_scan.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r6l.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_r6l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/cold_query.py --arms "hm:FLS_PIN_ARENA_MB=0;arena:FLS_PIN_ARENA_MB=8192" --runs 3 > $O/cold_query_r6l.txt 2>&1; echo "cold rc=$?"; tail -12 $O/cold_query_r6l.txt
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,sc1,nts --workload lineitem_full --scale 12.5 --rounds 6 --verify > $O/ab_builds_cpol_sf12_r6l.txt 2>&1; echo "ab sf12 rc=$?"; tail -2 $O/ab_builds_cpol_sf12_r6l.txt
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,sc1,nts --workload c3 --scale 1 --rounds 6 > $O/ab_builds_cpol_c3_r6l.txt 2>&1; echo "ab c3 rc=$?"; tail -2 $O/ab_builds_cpol_c3_r6l.txt
