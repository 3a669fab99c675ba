# decode-rated placement candidates: outputs only vs + FSST heaps vs + image copy vs both (bench command, interleaved processes)
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
B="python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic --no-verify"
for sc in 100 12.5; do
  for i in 1 2; do
    for arm in base heaps image both; do
      case $arm in base) E="";; heaps) E="FLS_PLACEMENT_HEAPS=1";; image) E="FLS_PLACEMENT_IMAGE=1";; both) E="FLS_PLACEMENT_HEAPS=1 FLS_PLACEMENT_IMAGE=1";; esac
      env $E timeout -k 10 300 $B --scale $sc > $O/abcand_sf${sc}_${arm}_$i.json 2> $O/abcand_sf${sc}_${arm}_$i.log || exit 1
      python3 -c "import json;d=json.load(open('$O/abcand_sf${sc}_${arm}_$i.json'));print('sf$sc $arm run $i', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
    done
  done
done
