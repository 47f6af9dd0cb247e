#!/bin/bash
# A GPU call of round 3: parity subset (PYTEST_K), then A/B of build_variants (VARIANTS) on
# BENCH_ARGS, then optional bench legs (r03_session.sh).  Each step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  mkdir -p gpurun_out/${TAG:-r03}
  echo "== pytest -k $PYTEST_K"
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "$PYTEST_K" > gpurun_out/${TAG:-r03}/pytest.txt 2>&1
  rc=$?; tail -5 gpurun_out/${TAG:-r03}/pytest.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then
  echo "== ab ($BENCH_ARGS)"; bash scripts/ab_variants.sh || exit 1
fi
if [ -n "$BENCH_LEGS" ]; then
  PYTEST_K= bash scripts/r03_session.sh || exit 1
fi
exit 0
