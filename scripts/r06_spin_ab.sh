#!/bin/bash
# A/B of the ring's wait (blocking vs KBZ_RING_SPIN=1 polling) on the plugin legs, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/spin
for r in 1 2; do
  for sp in 0 1; do
    for m in afl dynamorio; do
      KBZ_RING_SPIN=$sp timeout -k 10 300 python bench.py --workload plugin --mode $m --no-cpu \
        > gpurun_out/spin/${m}_spin${sp}_$r.json 2> gpurun_out/spin/${m}_spin${sp}_$r.err || { echo "$m $sp failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/spin/${m}_spin${sp}_$r.json').read().strip().splitlines()[-1]); print('$m spin=$sp run $r', d['us_per_exec_by_batch'])"
    done
  done
done
