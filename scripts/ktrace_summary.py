#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace of a bench.py run (run with --no-variants, so its last
STEPS pass-1 dispatches are the timed steps) next to the JSON line that same run printed:
the trace's pass-1 average, the fraction of 8 TB/s it gives, and the line's own HIP-event
figures.  Usage: ktrace_summary.py PROFDIR BENCH_LINE_FILE OUT_JSON"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import HBM_PEAK_GBS, summarize_ktrace  # noqa: E402

prof, line_file, dest = sys.argv[1:4]
line = json.loads([l for l in open(line_file) if l.startswith("{")][-1])
steps = line["steps"]
got = summarize_ktrace(glob.glob(os.path.join(prof, "**", "*kernel_trace.csv"), recursive=True),
                       steps)
if got is None:
    raise SystemExit("trace holds fewer pass-1 dispatches than the run's steps")
summ, per_step, durs = got
alg = line["roofline"]["algorithmic_bytes_per_launch"]
summ["frac_from_trace"] = round(alg / (summ["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
summ["line"] = {k: line.get(k) for k in ("value", "ms_per_step", "pass1_share_of_step")}
summ["line"]["hip_event_avg_launch_ms"] = line["roofline"]["avg_launch_ms"]
summ["line"]["frac"] = line["roofline"]["frac"]
summ["trace_vs_line_frac"] = round(summ["frac_from_trace"] / line["roofline"]["frac"], 4)
summ["trace_avg_le_ms_per_step"] = summ["avg_ms"] <= line["ms_per_step"]
summ["what"] = ("rocprofv3 --kernel-trace of the bench.py run itself (same process, same timed "
                f"dispatches): the last {steps} pass-1 dispatches; `line` = that run's JSON line")
json.dump(dict(summ, pass1_durations_ms=[round(x, 5) for x in durs], steps=per_step),
          open(dest, "w"), indent=1)
print(json.dumps({k: v for k, v in summ.items() if k != "what"}))
