#!/bin/bash
# Timing-only ablation of pass 1 (library must be built with KBZ_HIPCC_FLAGS=-DKBZ_ABLATION).
# KBZ_ABL: 0 = full kernel, 1 = no transform work, 2 = no hash chains, 3 = neither.
# KBZ_DEPTH: register prefetch ring depth (2, 3, 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for d in ${DEPTHS:-2 3 4}; do
  for a in ${ABLS:-0 3}; do
    KBZ_DEPTH=$d KBZ_ABL=$a timeout -k 10 300 python bench.py --no-cpu --no-pmc --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/abl_${d}_$a.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_${d}_$a.log').read().strip().splitlines()[-1]); print('DEPTH=$d ABL=$a pass1 ms', d['roofline']['avg_launch_ms'], 'GB/s', d['roofline']['achieved'], 'step ms', d['ms_per_step'])"
  done
done
