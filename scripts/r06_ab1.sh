cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/r06_ab
( while sleep 30; do date +%T >> gpurun_out/r06_ab/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== depth A/B config2 $(date +%T)"
STEPS=10 VARIANTS="base d3 d3e0 d4e0 base2 d3_2 d3e0_2" timeout -k 10 900 bash scripts/ab_variants.sh > gpurun_out/r06_ab/ab_depth.txt 2>&1; rc=$?; cat gpurun_out/r06_ab/ab_depth.txt; [ $rc -eq 0 ] || exit 1
echo "== k_fin A/B config3 novelty $(date +%T)"
VARIANTS="base fin1024 fin2048 win32 base2" NOV_ARGS="3 dynamorio config3" timeout -k 10 900 bash scripts/ab_novelty_trace.sh > gpurun_out/r06_ab/ab_fin_c3.txt 2>&1; rc=$?; cat gpurun_out/r06_ab/ab_fin_c3.txt; [ $rc -eq 0 ] || exit 1
