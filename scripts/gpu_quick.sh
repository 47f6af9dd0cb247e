#!/bin/bash
# Quick GPU session: selected parity tests (PYTEST_K), then timing variants (VARIANTS) on a
# workload (BENCH_ARGS), then per-wave stamps of a -DKBZ_STAMPS build (STAMPS).  First failure
# ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  echo "== pytest -k $PYTEST_K"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then
  echo "== ab"; bash scripts/ab_variants.sh || exit 1
fi
for v in $STAMPS; do
  echo "== stamps $v"
  KBZ_HIP_LIB=$PWD/build_variants/$v/libkbz_hip.so timeout -k 10 200 python tools/stamps_wide.py > gpurun_out/stamps_$v.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/stamps_$v.txt; [ $rc -eq 0 ] || exit $rc
done
