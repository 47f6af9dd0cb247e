#!/bin/bash
# Timing-only variants of libkbz_hip.so for A/B runs (scripts/ab_variants.sh); never used for
# results.  usage: build_variants.sh name:"-DFLAG ..." ...   -> build_variants/<name>/libkbz_hip.so
cd "$(dirname "$0")/.." || exit 1
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_variants/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
    -I include -I killerbeez_amd/csrc $flags killerbeez_amd/csrc/kbz_triage.hip \
    killerbeez_amd/csrc/kbz_set.hip killerbeez_amd/csrc/kbz_ipt.hip \
    -o build_variants/$name/libkbz_hip.so &
done
wait
ls -la build_variants/*/libkbz_hip.so
