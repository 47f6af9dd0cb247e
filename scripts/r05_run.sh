#!/bin/bash
# Round-5 GPU call: optional pytest selection, bench legs, and "direct" legs -- bench.py run
# under rocprofv3 --kernel-trace --stats itself, so the traced pass-1 dispatches are the ones
# its JSON line timed (scripts/ktrace_summary.py compares them).  Every GPU step has its own
# time limit; the first failure ends the call.
#   TAG=name TESTS="tests/test_rccl.py ..." KEXPR="pytest -k expression" LEGS="name|args;..."
#   DIRECT="name|args;..."
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  step "pytest $TESTS"
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
fi
if [ -n "$SMOKE" ]; then
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
if [ -n "$LEGS" ]; then
  IFS=';' read -ra L <<< "$LEGS"
  for leg in "${L[@]}"; do
    name=${leg%%|*}; args=${leg#*|}
    step "bench $name ($args)"
    KBZ_BENCH_KTRACE_OUT=$O/ktrace_$name.json timeout -k 10 ${LEG_LIMIT:-420} python -u bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
    tail -c 400 $O/bench_$name.json; echo
  done
fi
if [ -n "$DIRECT" ]; then
  IFS=';' read -ra L <<< "$DIRECT"
  for leg in "${L[@]}"; do
    name=${leg%%|*}; args=${leg#*|}
    step "direct $name ($args)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- python3 bench.py --no-pmc --no-ktrace --no-variants --no-cpu $args > $O/direct_$name.json 2> $O/direct_$name.err || { tail -20 $O/direct_$name.err; exit 1; }
    python3 scripts/ktrace_summary.py $O/prof_$name $O/direct_$name.json $O/direct_ktrace_$name.json || exit 1
    f=$(find $O/prof_$name -name '*kernel_stats.csv' | head -1); cp "$f" $O/direct_kernel_stats_$name.csv
    rm -f $(find $O/prof_$name -name '*kernel_trace.csv')
  done
fi
if [ -n "$AB" ]; then
  step "ab $AB ($AB_ARGS)"
  STEPS=${AB_STEPS:-10} VARIANTS="$AB" BENCH_ARGS="$AB_ARGS" timeout -k 10 900 bash scripts/ab_variants.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
if [ -n "$AB2" ]; then
  step "ab2 $AB2 ($AB2_ARGS)"
  STEPS=${AB_STEPS:-10} VARIANTS="$AB2" BENCH_ARGS="$AB2_ARGS" timeout -k 10 900 bash scripts/ab_variants.sh > $O/ab2.txt 2>&1 || { cat $O/ab2.txt; exit 1; }
  cat $O/ab2.txt
fi
if [ -n "$STAMPS" ]; then
  step stamps
  KBZ_HIP_LIB=$PWD/build_variants/stamps/libkbz_hip.so timeout -k 10 200 python tools/stamps.py > $O/stamps_k_pass1s.txt 2>&1 || { tail $O/stamps_k_pass1s.txt; exit 1; }
  cat $O/stamps_k_pass1s.txt
fi
if [ -n "$TAILST" ]; then
  step tailstamps
  KBZ_TAIL_NOVELTY=${TAILST_NOVELTY:-0} KBZ_TAIL_BATCHES=${TAILST_BATCHES:-16} KBZ_HIP_LIB=$PWD/build_variants/tailst/libkbz_hip.so timeout -k 10 300 python tools/tail_stamps.py > $O/tail_stamps.txt 2>&1 || { tail $O/tail_stamps.txt; exit 1; }
  tail -4 $O/tail_stamps.txt
fi
if [ -n "$NOVTRACE" ]; then  # NOVTRACE="name|STEPS MODE WORKLOAD;..." (tools/novelty_trace.py)
  IFS=';' read -ra L <<< "$NOVTRACE"
  for leg in "${L[@]}"; do
    name=${leg%%|*}; args=${leg#*|}
    step "noveltytrace $name ($args)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nov_$name -o run -- python3 tools/novelty_trace.py $args > $O/novelty_trace_$name.json 2> $O/novelty_trace_$name.err || { tail $O/novelty_trace_$name.err; exit 1; }
    python3 scripts/ktrace_kernels.py $O/prof_nov_$name > $O/novelty_kernels_$name.json || exit 1
    rm -f $(find $O/prof_nov_$name -name '*kernel_trace.csv')
    cat $O/novelty_trace_$name.json
  done
fi
if [ -n "$PROBE" ]; then
  step l2probe
  timeout -k 10 120 ./tools/l2_handoff_probe 1024 20 > $O/l2_handoff_probe.txt 2>&1 || { tail $O/l2_handoff_probe.txt; exit 1; }
  cat $O/l2_handoff_probe.txt
fi
if [ -n "$SQ" ]; then
  step "sq ($SQ_ARGS)"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --no-ktrace --no-variants $SQ_ARGS > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
  f=$(find $O/sq -name '*counter_collection.csv' | head -1); grep k_pass1 "$f" > $O/sq_pass1.csv; rm -rf $O/sq
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --no-ktrace --no-variants $SQ_ARGS > $O/sq2.log 2>&1 && { f=$(find $O/sq2 -name '*counter_collection.csv' | head -1); grep k_pass1 "$f" > $O/sq2_pass1.csv; rm -rf $O/sq2; }
fi
for f in $(find $O -name '*.stamp' 2>/dev/null); do rm -f $f; done
step done
