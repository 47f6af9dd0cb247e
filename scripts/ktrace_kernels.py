#!/usr/bin/env python3
"""Per-step kernel list of a rocprofv3 --kernel-trace directory (every pass-1 dispatch starts a
step): for each step the kernels with their start (us after that step's pass 1) and duration,
plus the mean duration per kernel name.  Usage: ktrace_kernels.py PROFDIR [STEPS]"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import summarize_ktrace  # noqa: E402

prof = sys.argv[1]
files = glob.glob(os.path.join(prof, "**", "*kernel_trace.csv"), recursive=True)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
if steps is None:  # every pass-1 dispatch
    import csv
    steps = sum(1 for f in files for r in csv.DictReader(open(f))
                if "::k_pass1" in r.get("Kernel_Name", ""))
got = summarize_ktrace(files, steps)
if got is None:
    raise SystemExit("no pass-1 dispatches")
summ, per_step, durs = got
mean = {}
for st in per_step:
    for k in st:
        mean.setdefault(k["kernel"], []).append(k["dur_us"])
summ["mean_dur_us"] = {k: round(sum(v) / len(v), 2) for k, v in mean.items()}
summ["steps"] = per_step
print(json.dumps(summ, indent=1))
