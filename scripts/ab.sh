#!/bin/bash
# A/B timing of library variants on one box: bench.py with KBZ_HIP_LIB=<variant>, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARIANTS:-build_variants/*.so}; do
    n=$(basename $v .so)
    KBZ_HIP_LIB=$v timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS_N:-20} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/ab_${n}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${n}_$rep.log').read().strip().splitlines()[-1]); print('$n rep $rep pass1 ms', d['roofline']['avg_launch_ms'], 'GB/s', d['roofline']['achieved'], 'step ms', d['ms_per_step'])"
  done
done
