#!/bin/bash
# A/B timing of libkbz_hip.so variants (build_variants/<name>/libkbz_hip.so) on one workload.
# usage (on the GPU box): VARIANTS="base nochain ..." BENCH_ARGS="--workload config3" ab_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-base}; do
  lib=build_variants/${v%_2}/libkbz_hip.so  # NAME_2: a second run of variant NAME
  case $v in base*) lib=killerbeez_amd/libkbz_hip.so;; esac
  KBZ_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-variants --no-pmc --steps ${STEPS:-6} \
    --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); print('$v', 'pass1 ms', d['roofline']['avg_launch_ms'], 'GB/s', d['roofline']['achieved'], 'step ms', d['ms_per_step'])"
done
