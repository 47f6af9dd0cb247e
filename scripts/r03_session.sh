#!/bin/bash
# One GPU session of round 3: optional parity subset (PYTEST_K), then bench legs (BENCH_LEGS:
# "name|args" entries separated by ';'), then an optional rocprofv3 kernel-stats pass (PROF_ARGS).
# Every GPU step has its own time limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p "$OUT"
if [ -n "$PYTEST_K" ]; then
  echo "== pytest -k $PYTEST_K"
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest.txt" 2>&1
  rc=$?; tail -5 "$OUT/pytest.txt"; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra LEGS <<< "$BENCH_LEGS"
for leg in "${LEGS[@]}"; do
  [ -z "$leg" ] && continue
  name=${leg%%|*}; args=${leg#*|}
  echo "== bench $name: $args"
  timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py $args > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  rc=$?; tail -c 1500 "$OUT/bench_$name.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/bench_$name.err"; exit $rc; }
done
if [ -n "$PROF_ARGS" ]; then
  echo "== rocprofv3 --kernel-trace --stats: $PROF_ARGS"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 bench.py $PROF_ARGS > "$OUT/prof.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -20 "$OUT/prof.log"; exit $rc; }
  f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && head -12 "$OUT/kernel_stats.csv"
fi
exit 0
