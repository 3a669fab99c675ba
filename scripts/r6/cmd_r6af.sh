# confirmation: decode-rated candidates with outputs only vs outputs + heaps + image copy, SF100, 4 interleaved runs
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
B="python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic --no-verify"
for i in 1 2 3 4; do
  for arm in base both; do
    case $arm in base) E="";; both) E="FLS_PLACEMENT_HEAPS=1 FLS_PLACEMENT_IMAGE=1";; esac
    env $E timeout -k 10 300 $B --scale 100 > $O/abcand2_${arm}_$i.json 2> $O/abcand2_${arm}_$i.log || exit 1
    python3 -c "import json;d=json.load(open('$O/abcand2_${arm}_$i.json'));print('sf100 $arm run $i', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
