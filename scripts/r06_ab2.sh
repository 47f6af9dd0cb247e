cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/r06_ab
( while sleep 30; do date +%T >> gpurun_out/r06_ab/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== k_fin A/B config3 novelty $(date +%T)"
VARIANTS="${VARIANTS:-base fin1024 fin2048 win32 base_2}" NOV_ARGS="${NOV_ARGS:-3 dynamorio config3}" timeout -k 10 1000 bash scripts/ab_novelty_trace.sh > gpurun_out/r06_ab/ab_${TAG:-fin_c3}.txt 2>&1; rc=$?; cat gpurun_out/r06_ab/ab_${TAG:-fin_c3}.txt; [ $rc -eq 0 ] || exit 1
