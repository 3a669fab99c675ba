# placement rating modes at bench level, interleaved processes: write probe (FLS_PLACEMENT_DECODE=0) vs decode rating (6 sets)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
B="python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic --no-verify"
for sc in 12.5 25 100; do
  for i in 1 2 3; do
    for arm in 0 6; do
      FLS_PLACEMENT_DECODE=$arm timeout -k 10 300 $B --scale $sc > $O/abmode_sf${sc}_d${arm}_$i.json 2> $O/abmode_sf${sc}_d${arm}_$i.log || exit 1
      python3 -c "import json;d=json.load(open('$O/abmode_sf${sc}_d${arm}_$i.json'));print('sf$sc decode=$arm run $i', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
    done
  done
done
