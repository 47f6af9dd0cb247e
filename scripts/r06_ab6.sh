#!/bin/bash
# Round 6: window items without the lanes that hold no new bit (KBZ_WIN_LANEMASK) -- claim-path
# parity, then A/B against nolm on novelty-heavy config 3 / config 2; then the plugin A/B.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06_ab6; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== pytest claims $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tail.py -m gpu -x -q --timeout 300 --timeout-method thread -k "claims or window or novelty or fresh or crash_hang or tail or uniform_density or full_size_config3" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
echo "== lanemask novelty config3 $(date +%T)"
VARIANTS="base nolm base_2 nolm_2" NOV_ARGS="3 dynamorio config3" timeout -k 10 700 bash scripts/ab_novelty_trace.sh > $O/ab_lanemask_c3.txt 2>&1; rc=$?; cat $O/ab_lanemask_c3.txt; [ $rc -eq 0 ] || exit 1
echo "== lanemask novelty config2 $(date +%T)"
VARIANTS="base nolm base_2 nolm_2" NOV_ARGS="5 dynamorio config2" timeout -k 10 500 bash scripts/ab_novelty_trace.sh > $O/ab_lanemask_c2.txt 2>&1; rc=$?; cat $O/ab_lanemask_c2.txt; [ $rc -eq 0 ] || exit 1
echo "== plugin A/B $(date +%T)"
timeout -k 10 600 bash scripts/r06_ab5.sh || exit 1
