#!/bin/bash
# Kernel-trace A/B of library variants: bench.py config 2 under rocprofv3 --kernel-trace, mean
# duration of every kernel over the timed steps.  usage (GPU box): VARIANTS="new prev" ab_ktrace.sh
# (a variant "name@VAR=value" runs the product library with that environment setting)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/abk; mkdir -p $O
for r in $(seq 1 ${REPS:-1}); do
for v in ${VARIANTS:-new}; do
  lib=killerbeez_amd/libkbz_hip.so; [ -f build_variants/$v/libkbz_hip.so ] && lib=build_variants/$v/libkbz_hip.so
  envv=""; case $v in *@*) envv=${v#*@}; v=${v%%@*};; esac
  [ -n "$envv" ] && export "$envv"
  rm -rf $O/prof_${v}_$r
  KBZ_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_${v}_$r -o run -- python3 bench.py --no-pmc --no-ktrace --no-variants --no-cpu --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
  python3 scripts/ktrace_kernels.py $O/prof_${v}_$r ${STEPS:-20} > $O/k_${v}_$r.json || exit 1
  python3 -c "
import json; k=json.load(open('$O/k_${v}_$r.json')); d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1])
print('$v', $r, 'step', d['ms_per_step'], 'span', k['median_step_span_ms'], 'mean_us', k['mean_dur_us'])"
  rm -rf $O/prof_${v}_$r
  [ -n "$envv" ] && unset "${envv%%=*}"
done
done
