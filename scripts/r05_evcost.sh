#!/bin/bash
# Cost of the pass-1 HIP events in the timed steps: the same config-2 run with and without them
# (KBZ_BENCH_P1_TIMING=0: no roofline), alternated.
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${TAG:-r05_ev}; mkdir -p $O
for i in 1 2 3; do
  for ev in 1 0; do
    KBZ_BENCH_P1_TIMING=$ev timeout -k 10 200 python bench.py --no-cpu --no-variants --no-pmc --no-ktrace --steps 20 > $O/ev${ev}_$i.json 2>/dev/null || exit 1
    echo "events=$ev run $i: $(python3 -c "import json;d=json.loads(open('$O/ev${ev}_$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
  done
done
