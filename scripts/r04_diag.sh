#!/bin/bash
# Round-4 diagnosis call: the golden triage tests through the staged tail, then the fused tail,
# each in its own process under a short limit (the first stops the call if it fails).
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_diag}; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== staged $(date +%T)"
KBZ_DEBUG_STAGED=1 timeout -k 10 240 python -u -m pytest tests/test_golden.py -m gpu -x -v --timeout 60 --timeout-method thread -k "${PYTEST_K:-test_triage_gpu}" > $O/staged.txt 2>&1 || { grep -E "PASS|FAIL|Timeout|Error" $O/staged.txt | head -20; exit 1; }
grep -cE "PASSED" $O/staged.txt
echo "== fused $(date +%T)"
timeout -k 10 240 python -u -m pytest tests/test_golden.py -m gpu -x -v --timeout 60 --timeout-method thread -k "${PYTEST_K:-test_triage_gpu}" > $O/fused.txt 2>&1 || { grep -E "PASS|FAIL|Timeout|Error" $O/fused.txt | head -20; exit 1; }
grep -cE "PASSED" $O/fused.txt
