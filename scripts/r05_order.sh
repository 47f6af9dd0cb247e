#!/bin/bash
# Is a process's pass-1 time set by what ran on the box before it?  Bench runs in sequence with
# GPU temperature / clock snapshots between them.
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/order; mkdir -p $O
snap() { (rocm-smi --showtemp --showclocks --showpower 2>/dev/null | grep -E "^(GPU|0 )|Temp|sclk|mclk|fclk|Power" | head -20) > $O/smi_$1.txt; }
run() { # name args
  snap $1
  timeout -k 10 300 python bench.py --no-cpu --no-variants $2 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', 'step', d['ms_per_step'], 'pass1', d['roofline']['avg_launch_ms'])"
}
run a1 "--no-pmc --no-ktrace"
run b1 ""
run a2 "--no-pmc --no-ktrace"
run a3 "--no-pmc --no-ktrace"
snap end
