# the e2e block run in its own process before the metric's upload (bench.py e2e_child)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
B="python3 bench.py --steps 5 --cpu-seconds 0 --no-traffic --no-verify"
for i in 1 2; do
  for arm in dec none; do
    case $arm in dec) E="";; none) E="FLS_PLACEMENT_DECODE=0 FLS_PLACEMENT_TRIES=1";; esac
    env $E timeout -k 10 400 $B > $O/abe2e3_${arm}_$i.json 2> $O/abe2e3_${arm}_$i.log || exit 1
    python3 -c "import json;d=json.load(open('$O/abe2e3_${arm}_$i.json'));e=d['e2e'];print('$arm run $i', round(d['ms_per_step'],3), 'engine', round(e['engine_scan_rows_s']/1e6), 'dc16', round(e['datachunk_rows_s_16t']/1e6), 'dc1', round(e['datachunk_rows_s_1t']/1e6), 'cold', round(e['datachunk_cold_rows_s_16t']/1e6))"
  done
done
