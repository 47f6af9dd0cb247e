#!/bin/bash
# Round-5 GPU call: optional pytest selection, bench legs, and "direct" legs -- bench.py run
# under rocprofv3 --kernel-trace --stats itself, so the traced pass-1 dispatches are the ones
# its JSON line timed (scripts/ktrace_summary.py compares them).  Every GPU step has its own
# time limit; the first failure ends the call.
#   TAG=name TESTS="tests/test_rccl.py ..." LEGS="name|args;..." DIRECT="name|args;..."
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  step "pytest $TESTS"
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
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
for f in $(find $O -name '*.stamp' 2>/dev/null); do rm -f $f; done
step done
