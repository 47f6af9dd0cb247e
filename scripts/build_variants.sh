#!/bin/bash
# Experiment builds of libkbz_hip.so for A/B runs (scripts/ab_variants.sh) and diagnostics
# (KBZ_STAMPS); never used for results, never the shipped library.
# usage: build_variants.sh name:"-DFLAG ..." ...   -> build_variants/<name>/libkbz_hip.so
# Each reports its flags through kbz_build_flags().  A spec may start with "--patch FILE" (a diff
# against killerbeez_amd/csrc applied to a copy, e.g. tools/ab_p1s.patch: the timing-only
# k_pass1s ablations, -DKBZ_AB_P1S=N; wrong results, never in the product tree).
cd "$(dirname "$0")/.." || exit 1
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  python3 -m killerbeez_amd.build --variant "$name" $flags &
done
wait
ls -la build_variants/*/libkbz_hip.so
