#!/bin/bash
# Round-2 measurement session on the gpurun box: default bench (config 2, fresh batches),
# the other workloads, a rocprofv3 kernel trace of config 2 and a live-PMC bench run.
# Every GPU step has its own time limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -c 3000 $OUT/$name.log | tail -3
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
}
for s in ${STEPS:-bench plugin merge stream prof pmc}; do
  case $s in
    bench)  run bench 600 python bench.py ;;
    plugin) run plugin 300 python bench.py --workload plugin ;;
    merge)  run merge 300 python bench.py --workload merge ;;
    stream) run stream 300 python bench.py --workload stream --steps 40 ;;
    config3) run config3 600 python bench.py --workload config3 --steps 10 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
              -- python3 bench.py --no-cpu --no-pmc ;;
    pmc)    run pmc 600 python bench.py --no-cpu --no-variants --steps 10 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
