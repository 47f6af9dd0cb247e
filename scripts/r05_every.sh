#!/bin/bash
# config 2 with the pass-1 events on every timed launch vs one in 4, alternated
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${TAG:-r05_every}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_timing.py -m gpu -x -q --timeout 120 > $O/pytest_timing.txt 2>&1 || { tail $O/pytest_timing.txt; exit 1; }
tail -1 $O/pytest_timing.txt
for i in 1 2 3; do
  for e in 1 4; do
    KBZ_BENCH_P1_EVERY=$e timeout -k 10 200 python bench.py --no-cpu --no-variants --no-pmc --no-ktrace --steps 20 > $O/e${e}_$i.json 2>/dev/null || exit 1
    echo "every=$e run $i: $(python3 -c "import json;d=json.loads(open('$O/e${e}_$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['timed_launches'])")"
  done
done
