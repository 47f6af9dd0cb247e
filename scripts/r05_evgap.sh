#!/bin/bash
# Gaps the pass-1 timing events leave around k_pass1s: the headline bench under
# rocprofv3 --kernel-trace with the product's event flags, two other flag choices and no events.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_evgap}; mkdir -p $O
for v in ${EVGAP_VARIANTS:-base evdef evnf noev}; do
  lib=$PWD/build_variants/$v/libkbz_hip.so; ev=1
  case $v in base) lib=$PWD/killerbeez_amd/libkbz_hip.so;; noev) lib=$PWD/killerbeez_amd/libkbz_hip.so; ev=0;; esac
  KBZ_BENCH_P1_TIMING=$ev KBZ_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p_$v -o run -- python3 bench.py --no-pmc --no-ktrace --no-variants --no-cpu > $O/line_$v.json 2>/dev/null || exit 1
  python3 scripts/ktrace_kernels.py $O/p_$v 20 > $O/k_$v.json || exit 1
  rm -rf $O/p_$v
  python3 - <<PY
import json
d=json.load(open("$O/k_$v.json")); st=d["steps"]
g=[s[1]["start_us"]-s[0]["dur_us"] for s in st if len(s)>1]
line=json.loads(open("$O/line_$v.json").read().strip().splitlines()[-1])
print("$v", "span", d["median_step_span_ms"], "pass1", d["median_ms"], "gap after pass1 us", round(sorted(g)[len(g)//2],2), "ms_per_step", line["ms_per_step"], "p1 events", line["roofline"]["avg_launch_ms"])
PY
done
