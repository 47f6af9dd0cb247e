#!/bin/bash
# Round 6: pass-1 writes before the next prefetch loads (k_pass1d, k_pass1n) -- parity of the
# pass-1 kernels, then A/B against the previous order (build_variants/wbefore) on novelty-heavy
# config 3 / AFL and on fresh config 3.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06_ab3; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "uniform_density or map_sizes or crash_hang or all_hang or at_scale or full_size_config3 or small_batches" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
echo "== novelty config3 $(date +%T)"
VARIANTS="base wbefore base_2 wbefore_2" NOV_ARGS="3 dynamorio config3" timeout -k 10 1000 bash scripts/ab_novelty_trace.sh > $O/ab_novelty_c3.txt 2>&1; rc=$?; cat $O/ab_novelty_c3.txt; [ $rc -eq 0 ] || exit 1
echo "== novelty afl $(date +%T)"
VARIANTS="base wbefore base_2 wbefore_2" NOV_ARGS="5 afl config2" timeout -k 10 600 bash scripts/ab_novelty_trace.sh > $O/ab_novelty_afl.txt 2>&1; rc=$?; cat $O/ab_novelty_afl.txt; [ $rc -eq 0 ] || exit 1
echo "== fresh config3 $(date +%T)"
STEPS=6 VARIANTS="base wbefore base_2 wbefore_2" BENCH_ARGS="--workload config3" timeout -k 10 900 bash scripts/ab_variants.sh > $O/ab_config3.txt 2>&1; rc=$?; cat $O/ab_config3.txt; [ $rc -eq 0 ] || exit 1
echo "== T late prefetch, fresh config2 $(date +%T)"
STEPS=10 VARIANTS="base tlate tlate3 base_2 tlate_2 tlate3_2" timeout -k 10 900 bash scripts/ab_variants.sh > $O/ab_tlate_config2.txt 2>&1; rc=$?; cat $O/ab_tlate_config2.txt; [ $rc -eq 0 ] || exit 1
echo "== T late prefetch, novelty config2 $(date +%T)"
VARIANTS="base tlate tlate3 base_2 tlate_2" NOV_ARGS="5 dynamorio config2" timeout -k 10 900 bash scripts/ab_novelty_trace.sh > $O/ab_tlate_novelty_c2.txt 2>&1; rc=$?; cat $O/ab_tlate_novelty_c2.txt; [ $rc -eq 0 ] || exit 1
