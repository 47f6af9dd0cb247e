#!/bin/bash
# Diagnosis: one pytest selection through several builds (VARIANTS: "product" or names under
# build_variants/).  A test failure moves on to the next build; a time limit, abort or crash
# ends the call.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_variants}; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in ${VARIANTS:-product}; do
  lib=""; [ "$v" = product ] || lib=$PWD/build_variants/$v/libkbz_hip.so
  echo "== $v $(date +%T)"
  KBZ_HIP_LIB=$lib timeout -k 10 ${LIMIT:-240} python -u -m pytest ${TESTS:-tests/test_golden.py} -m gpu -v --timeout 90 --timeout-method thread -k "${PYTEST_K:-test_triage_gpu}" > $O/$v.txt 2>&1
  rc=$?
  grep -E "passed|failed" $O/$v.txt | tail -1
  grep -E "FAILED|Error:" $O/$v.txt | head -6
  case $rc in 124|137|134|139) echo "stop: rc=$rc"; exit $rc;; esac
done
