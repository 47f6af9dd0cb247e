#!/bin/bash
# Same-box A/B of the tail fusion: HEAD library + HEAD bench vs the working-tree library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  PYTHONPATH=. KBZ_HIP_LIB=build_variants/head.so timeout -k 10 300 python build_variants/bench_head.py --no-cpu --steps 30 --warmup 3 > gpurun_out/ab_head_$rep.log 2>&1 || exit $?
  KBZ_HIP_LIB=build_variants/tail.so timeout -k 10 300 python bench.py --no-cpu --steps 30 --warmup 3 > gpurun_out/ab_tail_$rep.log 2>&1 || exit $?
  for v in head tail; do python3 -c "import json; d=json.loads(open('gpurun_out/ab_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v rep $rep step ms', d['ms_per_step'], 'pass1 ms', d['roofline']['avg_launch_ms'], 'value', d['value'])"; done
done
