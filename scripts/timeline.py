#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 --kernel-trace CSV of bench.py (one step = one
pass-1 launch and the launches after it).  usage: timeline.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import sys


def steps(path):
    tr = list(csv.DictReader(open(path)))
    ours = [r for r in tr if "(anonymous namespace)::k_" in r["Kernel_Name"]]
    ours.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for r in ours:
        k = r["Kernel_Name"].split("(anonymous namespace)::")[1].split("(")[0].split("<")[0]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if k.startswith("k_pass1"):
            out.append({"_start": int(r["Start_Timestamp"])})
        if out:
            out[-1][k] = round(out[-1].get(k, 0) + d, 2)
            out[-1]["_end"] = int(r["End_Timestamp"])
    for i, s in enumerate(out):
        s["span_us"] = round((s["_end"] - s["_start"]) / 1e3, 2)
    return [{k: v for k, v in s.items() if not k.startswith("_")} for s in out]


if __name__ == "__main__":
    st = steps(sys.argv[1])
    for i, s in enumerate(st):
        print(i, " ".join(f"{k}={v}" for k, v in s.items()))
    if len(sys.argv) > 2:
        json.dump({"steps": st}, open(sys.argv[2], "w"), indent=0)
