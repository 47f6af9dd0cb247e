#!/bin/bash
# One GPU session on the gpurun box: parity tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults, aborts, segfaults or times out (rc >= 2 from pytest,
# any nonzero rc from the others).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-tests bench prof}"
PYTEST_ARGS="${PYTEST_ARGS:--m gpu -x -v --timeout 120 --timeout-method thread}"
for s in $STEPS; do
  case $s in
    tests)
      echo "== pytest $PYTEST_ARGS $(date +%T)"
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests $PYTEST_ARGS > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -25 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
      [ $rc -le 1 ] || exit $rc ;;
    smoke)
      echo "== smoke $(date +%T)"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -5 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      echo "== bench $(date +%T)"
      timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
      rc=$?; tail -3 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      echo "== rocprofv3 $(date +%T)"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
        -- python3 bench.py --steps 40 --warmup 2 --no-cpu --no-pmc ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
      rc=$?; tail -3 $OUT/prof.log; [ $rc -eq 0 ] || exit $rc
      find $OUT/prof -name "*stats*.csv" | head -5 ;;
    pmc)
      echo "== rocprofv3 pmc $(date +%T)"
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-pmc ${BENCH_ARGS:-} > $OUT/pmc1.log 2>&1
      rc=$?; tail -2 $OUT/pmc1.log; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-pmc ${BENCH_ARGS:-} > $OUT/pmc2.log 2>&1
      rc=$?; tail -2 $OUT/pmc2.log; [ $rc -eq 0 ] || exit $rc ;;
    sq)
      echo "== rocprofv3 SQ counters $(date +%T)"
      timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
        --output-format csv -d $OUT/sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-pmc ${BENCH_ARGS:-} > $OUT/sq.log 2>&1
      rc=$?; tail -2 $OUT/sq.log; [ $rc -eq 0 ] || exit $rc ;;
    probe)
      echo "== bwprobe $(date +%T)"
      timeout -k 10 120 ./tools/bwprobe 4096 > $OUT/bwprobe.log 2>&1
      rc=$?; cat $OUT/bwprobe.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
