#!/bin/bash
# A/B of libkbz_hip.so variants on config 2: the fresh headline step and the novelty-heavy
# variant (all-0xff maps), same bench run.  usage (GPU box): VARIANTS="base rec8" ab_novelty.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abn
for v in ${VARIANTS:-base}; do
  lib=build_variants/${v%_2}/libkbz_hip.so
  case $v in base*) lib=killerbeez_amd/libkbz_hip.so;; esac
  KBZ_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-pmc --no-ktrace --steps ${STEPS:-20} \
    --warmup 5 ${BENCH_ARGS:-} > gpurun_out/abn/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abn/$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abn/$v.log').read().strip().splitlines()[-1]); nv=d['variants']['novelty_heavy']
print('$v', 'step', d['ms_per_step'], 'pass1', d['roofline']['avg_launch_ms'], 'novelty', nv['ms_per_step'], 'nov_pass1', nv['pass1_ms'], 'ratio', round(nv['ms_per_step']/d['ms_per_step'],3), 'stages', nv['stage_ms'])"
done
