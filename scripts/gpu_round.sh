#!/bin/bash
# GPU-box runner (the one script gpurun calls): every step under its own time
# limit, steps chained so the first failure ends the call.
#
#   bash scripts/gpu_round.sh <tag> <mode> [<mode> ...]
#
# modes:
#   test        full `pytest -m gpu` suite, then __graft_entry__.smoke()
#   pytest:<k>  the gpu tests matching -k <k>
#   bench       default bench (lineitem_full SF100, PMC traffic) + rocprofv3
#               kernel trace / stats of the same command
#   shares      per-GPU shares of the 4- and 8-GPU runs (SF25, SF12.5)
#   configs     bench lines of the other configurations (c3, c4, lineitem, lineitem_dbl)
#   percol      per-column rates, lineitem_full SF10
#   ab:<variants>:<workload>:<scale>:<cols>[:<rounds>]
#               interleaved same-process A/B of library builds (scripts/ab.py;
#               `base` = libflsgpu.so, `lab` = libflsgpu_lab.so ...)
#   abenv:<workload>:<scale>:<cols>:<arms>
#               same-buffer A/B of runtime knobs (scripts/ab_env.py; arms
#               name=ENV=V,ENV2=V2;name2=...)
#   fsstsq:<kernel>[:<scale>]  SQ counters of an FSST kernel on l_comment (3 PMC passes)
#   e2e         read_fastlanes DataChunk delivery, 1 and 16 threads, phase profile
#   e2earms:<arms>  the same with interleaved env arms (name:VAR=v,...;name2:...)
#   copy:<workload>:<scale>:<reps>:<arms>
#               COPY (read_fastlanes) TO (FORMAT fls), env arms interleaved
#               (scripts/writer_bench.py --copy-only; arms name:VAR=v,...;name2:...)
#   launcher2   bench.py --gpus 2 rehearsal (both ranks on the one GPU)
#   build:<t>   make <t> on the box (lab / exp / trace: the experiment and
#               timing libraries are not pushed, .gpurunignore)
#   wavetrace:<workload>:<scale>:<cols>[:<env>]  per-wave timeline of one
#               main decode launch (needs build:trace first)
# Results go to gpurun_out/<mode>_<tag>.*; copy what is judged to profiles/.
TAG=${1:?tag}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
PYT="python -u -m pytest tests -m gpu -q -rA -x -p no:cacheprovider --timeout 120 --timeout-method thread"
step() {  # step <timeout> <log> <cmd...>: run, report, stop the call on failure
    local t=$1 log=$2; shift 2
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    echo "[$TAG] $* -> rc=$rc ($(tail -1 "$log" | cut -c1-200))"
    return $rc
}
for mode in "$@"; do
  case "$mode" in
  test)
    step 600 $O/pytest_gpu_$TAG.log $PYT || exit $?
    step 300 $O/smoke_$TAG.log python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
  pytest:*)
    k=${mode#pytest:}
    step 600 $O/pytest_${k//[^A-Za-z0-9_]/_}_$TAG.log $PYT -k "$k" || exit $? ;;
  bench)
    timeout -k 10 500 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.log
    rc=$?; echo "[$TAG] bench rc=$rc"; cat $O/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
    step 400 $O/prof_$TAG.log rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o kt --output-format csv -- \
        python3 bench.py --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic || exit $?
    find $O/prof_$TAG -name "*kernel_stats.csv" -exec head -4 {} \;
    # per-step spans of the same trace (a step is several grids: the kernel
    # averages above are not a step) and the roofline fraction of their mean
    ab=$(python3 -c "import json;print(json.load(open('$O/bench_$TAG.json'))['roofline']['algo_bytes_per_launch'])")
    kt=$(find $O/prof_$TAG -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_span.py "$kt" --algo-bytes "$ab" > $O/step_spans_$TAG.txt && tail -2 $O/step_spans_$TAG.txt ;;
  shares)
    for sf in 25 12.5; do
      timeout -k 10 400 python bench.py --scale $sf --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic \
          > $O/bench_sf${sf}_$TAG.json 2> $O/bench_sf${sf}_$TAG.log
      rc=$?; python3 -c "import json;d=json.load(open('$O/bench_sf${sf}_$TAG.json'));print('sf$sf', d['ms_per_step'], d['roofline']['frac'])"
      [ $rc -eq 0 ] || exit $rc
    done
    # the 8-GPU share's kernel trace and step spans
    step 300 $O/prof_sf12_$TAG.log rocprofv3 --kernel-trace --stats -d $O/prof_sf12_$TAG -o kt --output-format csv -- \
        python3 bench.py --scale 12.5 --steps 20 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic || exit $?
    ab=$(python3 -c "import json;print(json.load(open('$O/bench_sf12.5_$TAG.json'))['roofline']['algo_bytes_per_launch'])")
    kt=$(find $O/prof_sf12_$TAG -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_span.py "$kt" --algo-bytes "$ab" > $O/step_spans_sf12_$TAG.txt && tail -2 $O/step_spans_sf12_$TAG.txt ;;
  configs)
    for wl in c3 c4 lineitem lineitem_dbl; do
      timeout -k 10 500 python bench.py --workload $wl --steps 10 --cpu-seconds 5 > $O/bench_${wl}_$TAG.json 2> $O/bench_${wl}_$TAG.log
      rc=$?; echo "[$TAG] bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 -c "import json;d=json.load(open('$O/bench_${wl}_$TAG.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['frac'],d['roofline']['traffic'])"
    done ;;
  percol)
    step 300 $O/percol_$TAG.txt python scripts/percol.py --workload lineitem_full --scale 10 || exit $? ;;
  ab:*)
    IFS=: read -r _ vars wl sc cols rounds <<< "$mode"
    step 600 $O/ab_${TAG}_${wl}_${sc}.txt python scripts/ab.py --variants "$vars" --workload "$wl" --scale "$sc" \
        --cols "$cols" --rounds "${rounds:-7}" || exit $?
    grep -v amdgpu.ids $O/ab_${TAG}_${wl}_${sc}.txt ;;
  abenv:*)
    IFS=: read -r _ wl sc cols arms <<< "$mode"
    step 600 $O/abenv_${TAG}_${wl}_${sc}.txt python scripts/ab_env.py --workload "$wl" --scale "$sc" --cols "$cols" \
        --arms $(echo "$arms" | tr ';' ' ') || exit $?
    grep -v amdgpu.ids $O/abenv_${TAG}_${wl}_${sc}.txt ;;
  fsstsq:*)   # fsstsq:<kernel substring>[:<scale>[:<cols>[:<workload>]]]: SQ counters of a kernel on l_comment (or cols), 3 PMC passes
    IFS=: read -r _ kern sc cols wl <<< "$mode"
    P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
    P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAVES"
    P3="SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"
    i=0
    for P in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      timeout -k 10 -s KILL 120 rocprofv3 --pmc $P -d $O/fsq_${TAG}_$i -o pmc --output-format csv -- \
          python3 scripts/fsst_prof.py --scale "${sc:-10}" --cols "${cols:-15}" --workload "${wl:-lineitem_full}" > $O/fsq_${TAG}_$i.log 2>&1
      rc=$?; echo "[$TAG] pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/fsq_${TAG}_$i.log; exit $rc; }
    done
    python3 scripts/pmc_summary.py "$kern" $O/fsq_${TAG}_1 $O/fsq_${TAG}_2 $O/fsq_${TAG}_3 | tee $O/fsst_sq_$TAG.txt ;;
  e2e)
    step 600 $O/e2e_phases_$TAG.txt python scripts/e2e_phases.py --scale 10 || exit $? ;;
  e2earms:*)  # e2earms:<arms>: interleaved env arms of the 16-thread DataChunk scan
    step 600 $O/e2e_arms_$TAG.txt python scripts/e2e_phases.py --scale 10 --arms "${mode#e2earms:}" || exit $? ;;
  e2eenv:*)  # e2eenv:<name>:<VAR=val,...>: the e2e phases with the env set for the whole process, 6 warm 16-thread queries
    IFS=: read -r _ nm kv <<< "$mode"
    step 600 $O/e2e_env_${TAG}_$nm.txt env FLS_SCAN_PROFILE=1 ${kv//,/ } python scripts/e2e_phases.py --scale 10 \
        --arms "q:" --reps 6 || exit $?
    grep "arm q" $O/e2e_env_${TAG}_$nm.txt ;;
  copy:*)  # copy:<workload>:<scale>:<reps>:<arms>: COPY (read_fastlanes) TO fls, env arms interleaved
    IFS=: read -r _ wl sc reps arms <<< "$mode"
    step 900 $O/copy_${TAG}_${wl}_${sc}.txt python scripts/writer_bench.py --copy-only --workload "$wl" \
        --scale "$sc" --reps "$reps" --arms "$arms" || exit $?
    grep median $O/copy_${TAG}_${wl}_${sc}.txt ;;
  build:*)
    step 600 $O/build_${mode#build:}_$TAG.log make -C duckdb-fastlane_amd -j16 "${mode#build:}" || exit $? ;;
  wavetrace:*)
    IFS=: read -r _ wl sc cols env <<< "$mode"
    step 300 $O/wave_trace_${TAG}_${wl}_${sc}.txt env FLS_LIB=libflsgpu_trace.so python scripts/wave_trace.py \
        --workload "$wl" --scale "$sc" --cols "$cols" --env "$env" --out $O/wave_trace_${TAG}.npz || exit $?
    head -20 $O/wave_trace_${TAG}_${wl}_${sc}.txt ;;
  launcher2)
    timeout -k 10 600 python bench.py --gpus 2 --scale 1 --steps 5 --cpu-seconds 0 --e2e-scale 0 --no-traffic \
        > $O/bench_gpus2_$TAG.json 2> $O/bench_gpus2_$TAG.log
    rc=$?; echo "[$TAG] launcher2 rc=$rc"; cat $O/bench_gpus2_$TAG.json; [ $rc -eq 0 ] || exit $rc ;;
  *)
    echo "unknown mode $mode"; exit 2 ;;
  esac
done
