#!/usr/bin/env python3
"""profiles/CURRENT.md from one evidence directory (the round's final build): ONE current number
per leg, each with the file it comes from.  README.md and DESIGN.md cite this table.

usage: current_table.py profiles/r06_final > profiles/CURRENT.md
"""
import json
import os
import re
import sys

D = sys.argv[1]


def load(name):
    p = os.path.join(D, name)
    if not os.path.exists(p):
        return None
    txt = open(p).read().strip()
    if not txt:
        return None
    try:
        return json.loads(txt)
    except json.JSONDecodeError:  # a bench log: the JSON line is the last one
        return json.loads(txt.splitlines()[-1])


def f(x, nd=1):
    return "—" if x is None else f"{x:,.{nd}f}"


def src(name):
    return f"`{os.path.join(D, name)}`"


rows = []
c2 = load("bench_config2.json")
if c2:
    r, v = c2["roofline"], c2["variants"]
    nov = v.get("novelty_heavy", {})
    sh = v.get("sharded_protocol_world1", {})
    tr = r.get("traffic")
    rows.append((
        "config 2: 65,536 sparse traces x 64 KiB, DynamoRIO, never-seen batches (headline)",
        f"**{c2['value'] / 1e6:.2f} M traces/s**, {c2['ms_per_step']:.4f} ms per step",
        f"pass 1 `{r['kernel']}` {r['avg_launch_ms']:.4f} ms = **{r['frac'] * 100:.1f} %** of 8 TB/s "
        f"(HIP events; child kernel trace {r.get('rocprof_frac', 0) * 100:.1f} %); PMC traffic "
        f"{tr / r['algorithmic_bytes_per_launch']:.4f}x algorithmic" if tr else "",
        src("bench_config2.json")))
    rows.append((
        "config 2 variants (same line)",
        f"steady state {v['steady_state_seen_batches']['ms_per_step']:.4f} ms; 90 % repeats "
        f"{v['repeats90']['ms_per_step']:.4f} ms; novelty-heavy {nov.get('ms_per_step', 0):.4f} ms "
        f"= {nov.get('ms_per_step', 0) / c2['ms_per_step']:.2f}x a fresh step",
        f"sharded protocol at world 1 (both RCCL all-gathers forced): "
        f"{sh.get('ms_per_step', 0):.4f} ms, +{sh.get('extra_us_per_step', 0):.1f} µs over the "
        f"fused step" if sh and "ms_per_step" in sh else "",
        src("bench_config2.json")))
    cb = c2.get("cpu_baseline", {})
    ca = c2.get("cpu_baseline_all_cores", {})
    rows.append((
        "config 2 on the host CPU",
        f"the reference's own DR loop: {f(cb.get('value'), 0)} traces/s on {cb.get('cores')} core "
        f"({c2['value'] / cb['value']:,.0f}x slower than the GPU)" if cb.get("value") else "—",
        f"the restatement's sharded decomposition: {f(ca.get('value'), 0)} traces/s on "
        f"{ca.get('cores')} threads" if ca.get("value") else "",
        src("bench_config2.json")))
dk = load("direct_ktrace_config2.json")
if dk:
    rows.append((
        "config 2, the bench run itself under rocprofv3 --kernel-trace",
        f"traced pass-1 avg {dk['avg_ms']:.4f} ms = {dk['frac_from_trace'] * 100:.1f} % of 8 TB/s",
        f"trace frac / line frac = {dk['trace_vs_line_frac']:.4f}", src("direct_ktrace_config2.json")))
c3 = load("bench_config3.json")
if c3:
    r, v = c3["roofline"], c3["variants"]
    nov = v.get("novelty_heavy", {})
    vi = r.get("valu_issue", {})
    rows.append((
        "config 3: 16,384 dense traces x 1 MiB",
        f"{c3['value'] / 1e6:.2f} M traces/s, {c3['ms_per_step']:.4f} ms per step; novelty-heavy "
        f"{nov.get('ms_per_step', 0):.3f} ms = {nov.get('ms_per_step', 0) / c3['ms_per_step']:.2f}x",
        f"`{r['kernel']}` {r['avg_launch_ms']:.4f} ms = {r['frac'] * 100:.1f} % of 8 TB/s; "
        f"{vi.get('frac', 0) * 100:.1f} % of its VALU-issue floor", src("bench_config3.json")))
for leg, name in (("afl", "AFL"), ("afl_classify", "AFL_CLASSIFY")):
    b = load(f"bench_{leg}.json")
    if b:
        r, v = b["roofline"], b["variants"]
        nov = v.get("novelty_heavy", {})
        rows.append((
            f"config-2 shape, {name} semantics (3 virgin maps, no hash: the AFL plugin)",
            f"{b['value'] / 1e6:.2f} M traces/s, {b['ms_per_step']:.4f} ms per step; novelty-heavy "
            f"{nov.get('ms_per_step', 0) / b['ms_per_step']:.2f}x",
            f"`{r['kernel']}` {r['frac'] * 100:.1f} % of 8 TB/s", src(f"bench_{leg}.json")))
m = load("bench_merge.json")
if m:
    r = m["roofline"]
    rows.append(("config 4: merger AND-fold of 100,000 x 192 KiB states",
                 f"{m['value'] / 1e6:.2f} M states/s", f"{r['frac'] * 100:.1f} % of 8 TB/s; PMC "
                 f"traffic {r['traffic'] / r['algorithmic_bytes_per_launch']:.4f}x"
                 if r.get("traffic") and r.get("algorithmic_bytes_per_launch") else
                 f"{r['frac'] * 100:.1f} % of 8 TB/s", src("bench_merge.json")))
s = load("bench_stream.json")
if s:
    md = s.get("multi_device_host_batch", {})
    md_txt = "; ".join(f"{k}: {v['frac_of_pinned_h2d_peak'] * 100:.0f} %" for k, v in md.items()
                       if isinstance(v, dict) and "frac_of_pinned_h2d_peak" in v)
    rows.append(("config 5: config-2 traces from host memory + unique crash/hang table",
                 f"{s['value'] / 1e6:.2f} M traces/s", f"{s['pcie_frac'] * 100:.0f} % of the "
                 f"pinned H2D peak of the same run; multi-device host batches: {md_txt}",
                 src("bench_stream.json")))
for leg, name in (("plugin", "dynamorio_gpu"), ("plugin_afl", "afl_gpu")):
    p = load(f"bench_{leg}.json")
    if p:
        by = p["us_per_exec_by_batch"]
        cb = p.get("cpu_baseline", {})
        rows.append((f"plugin `{name}`, µs per exec from C (batch 1 / 16 / 256 / 4,096)",
                     " / ".join(f(by.get(k), 2) for k in ("1", "16", "256", "4096")),
                     f"reference step on one core: {cb.get('us_per_exec', 0):.2f} µs",
                     src(f"bench_{leg}.json")))
pt = os.path.join(D, "pytest_gpu.txt")
if os.path.exists(pt):
    last = [l for l in open(pt).read().splitlines() if re.search(r"passed|failed", l)]
    rows.append(("`pytest -m gpu` on the final build", last[-1].strip("= ") if last else "—", "",
                 src("pytest_gpu.txt")))

print("# Current numbers (one per leg)\n")
print(f"Generated by `scripts/current_table.py {D}` from the final build's evidence run on one "
      "MI355X.  Boxes differ by up to ~10 % (clock) and runs on one box by ±2-3 %; the "
      "driver's own line is `BENCH_r06.json`.\n")
print("| leg | result | roofline / notes | file |")
print("|---|---|---|---|")
for a, b, c, d in rows:
    print(f"| {a} | {b} | {c} | {d} |")
