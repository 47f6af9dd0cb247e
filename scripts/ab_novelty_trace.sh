#!/bin/bash
# A/B of libkbz_hip.so variants on tools/novelty_trace.py (novelty-heavy steps on all-0xff maps,
# then fresh steps), no profiler: ms per step of each kind by HIP events.
# usage (GPU box): VARIANTS="base fin1024 ..." NOV_ARGS="3 dynamorio config3" ab_novelty_trace.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in ${VARIANTS:-base}; do
  lib=build_variants/${v%_2}/libkbz_hip.so  # NAME_2: a second run of variant NAME
  case $v in base*) lib=killerbeez_amd/libkbz_hip.so;; esac
  r=$(KBZ_HIP_LIB=$PWD/$lib timeout -k 10 300 python tools/novelty_trace.py ${NOV_ARGS:-3 dynamorio config3} 2>&1 | tail -1) || { echo "$v failed: $r"; exit 1; }
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$v', 'novelty', d['ms_per_step'], d['ms'], 'fresh', d['fresh_ms_per_step'], 'ratio', round(d['ms_per_step'] / d['fresh_ms_per_step'], 3))" "$r" || { echo "$v: $r"; exit 1; }
done
