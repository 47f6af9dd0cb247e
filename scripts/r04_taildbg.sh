#!/bin/bash
# Diagnosis: the golden AFL triage through a KBZ_TAIL_DEBUG build (k_tail printf, short spins),
# then through the product build; each under its own short limit.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_taildbg; mkdir -p $O
KBZ_HIP_LIB=$PWD/build_variants/taildbg/libkbz_hip.so timeout -k 10 120 python -u -m pytest tests/test_golden.py -m gpu -x -v -s --timeout 90 --timeout-method thread -k "${PYTEST_K:-test_triage_gpu and afl-0-narrow}" > $O/out.txt 2>&1
rc=$?
grep -c k_tail $O/out.txt
grep -E "PASS|FAIL|Error|assert" $O/out.txt | head -20
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_golden.py -m gpu -x -v --timeout 90 --timeout-method thread -k "${PYTEST_K2:-test_triage_gpu}" > $O/product.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|Timeout" $O/product.txt | head -20
exit $rc
