#!/bin/bash
# Round 6: k_fin permuted item order (finperm) on novelty-heavy config 3; the cost of pass 1's
# segment-OR atomics on config 2 (ab64: timing-only ablation, wrong results).
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06_ab4; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== finperm novelty config3 $(date +%T)"
VARIANTS="base finperm base_2 finperm_2" NOV_ARGS="3 dynamorio config3" timeout -k 10 700 bash scripts/ab_novelty_trace.sh > $O/ab_finperm_c3.txt 2>&1; rc=$?; cat $O/ab_finperm_c3.txt; [ $rc -eq 0 ] || exit 1
echo "== segment atomics ablation config2 $(date +%T)"
STEPS=10 VARIANTS="base ab64 base_2 ab64_2" BENCH_ARGS="--no-selfcheck" timeout -k 10 600 bash scripts/ab_variants.sh > $O/ab_segatomics_c2.txt 2>&1; rc=$?; cat $O/ab_segatomics_c2.txt; [ $rc -eq 0 ] || exit 1
