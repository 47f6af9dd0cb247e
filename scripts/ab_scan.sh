#!/bin/bash
# Same-box A/B: tail-fused library vs + segment skip in k_scan (both with the current bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for v in tail scan; do
    KBZ_HIP_LIB=build_variants/$v.so timeout -k 10 300 python bench.py --no-cpu --steps 30 --warmup 3 > gpurun_out/ab_${v}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v rep $rep step ms', d['ms_per_step'], 'pass1 ms', d['roofline']['avg_launch_ms'], 'value', d['value'])"
  done
done
