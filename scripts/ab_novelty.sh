#!/bin/bash
# A/B of libkbz_hip.so variants on the bench's novelty-heavy and cold-batch variants
# (VARIANTS, LEGS = bench argument sets separated by ';').  Timing only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abn
IFS=';' read -ra LG <<< "${LEGS:---mode dynamorio}"
for v in $VARIANTS; do
  for a in "${LG[@]}"; do
    tag=$(echo "$v $a" | tr -c 'a-z0-9' '_')
    KBZ_HIP_LIB=$PWD/build_variants/$v/libkbz_hip.so timeout -k 10 300 python bench.py --no-cpu --no-pmc --steps 6 --warmup 2 $a > gpurun_out/abn/$tag.log 2>&1 || { echo "$v $a failed"; tail -5 gpurun_out/abn/$tag.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abn/$tag.log').read().strip().splitlines()[-1]); v=d['variants']; nh=v.get('novelty_heavy',{}); print('$v', '$a', 'step', d['ms_per_step'], 'cold', v['cold_first_batch_ms'], 'novelty', nh.get('ms_per_step'), 'resolve', nh.get('stage_ms',{}).get('resolve'), 'claims', nh.get('claims_per_batch'))"
  done
done
