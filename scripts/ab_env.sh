#!/bin/bash
# A/B of run-time knobs (environment) on the product library, interleaved REPS times.
# usage (GPU box): ENVS="base|;in8|KBZ_DEBUG_TAIL_INLINE_MAX=8" REPS=2 ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abe
IFS=';' read -ra L <<< "${ENVS:-base|}"
for r in $(seq 1 ${REPS:-2}); do
  for e in "${L[@]}"; do
    name=${e%%|*}; vars=${e#*|}
    env $vars timeout -k 10 300 python bench.py --no-cpu --no-pmc --no-ktrace --steps ${STEPS:-20} --warmup 5 \
      ${BENCH_ARGS:---no-variants} > gpurun_out/abe/${name}_$r.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/abe/${name}_$r.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/abe/${name}_$r.log').read().strip().splitlines()[-1]); nv=d.get('variants',{}).get('novelty_heavy')
print('$name', $r, 'step', d['ms_per_step'], 'pass1', d['roofline']['avg_launch_ms'], 'rest', round(d['ms_per_step']-d['roofline']['avg_launch_ms'],4), ('novelty %s ratio %.3f' % (nv['ms_per_step'], nv['ms_per_step']/d['ms_per_step'])) if nv else '')"
  done
done
