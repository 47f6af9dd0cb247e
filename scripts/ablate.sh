#!/bin/bash
# Timing-only ablation of pass 1 (library must be built with KBZ_HIPCC_FLAGS=-DKBZ_ABLATION).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for a in 0 1 2 3 0; do
  KBZ_ABL=$a timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/abl_$a.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$a.log').read().strip().splitlines()[-1]); print('ABL=$a pass1 ms', d['roofline']['avg_launch_ms'], 'GB/s', d['roofline']['achieved'])"
done
