#!/bin/bash
# Round-4 evidence on one MI355X: full parity suite, smoke, every bench leg, rocprofv3 kernel
# stats (config 2, config 3) and one SQ-counter pass over config 3.  Each GPU step has its own
# time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_ev}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
IFS=';' read -ra LEGS <<< "${LEGS:-config2|;config3|--workload config3;merge|--workload merge;stream|--workload stream;plugin|--workload plugin;plugin_afl|--workload plugin --mode afl;afl|--mode afl;afl_classify|--mode afl_classify}"
for leg in "${LEGS[@]}"; do
  name=${leg%%|*}; args=${leg#*|}
  step "bench $name ($args)"
  KBZ_BENCH_KTRACE_OUT=$O/ktrace_$name.json timeout -k 10 400 python -u bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  tail -c 300 $O/bench_$name.json; echo
done
if [ -z "$SKIP_PROF" ]; then
  for w in config2 config3; do
    step "rocprofv3 $w"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-pmc --no-ktrace --no-variants > $O/prof_$w.log 2>&1 || { tail -20 $O/prof_$w.log; exit 1; }
    f=$(find $O/prof_$w -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$w.csv; head -4 $O/kernel_stats_$w.csv
  done
  step "sq counters config3"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu --no-pmc --no-ktrace --no-variants > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
  f=$(find $O/sq -name '*counter_collection.csv' | head -1); cp "$f" $O/sq_config3.csv; ls -la $O/sq_config3.csv
fi
step done
