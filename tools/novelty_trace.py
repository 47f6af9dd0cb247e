#!/usr/bin/env python3
"""Diagnostic (not the product): novelty-heavy steps for a rocprofv3 --kernel-trace run.
A warmed-up context triages STEPS never-seen batches (config 2: 65,536 x 64 KiB; config 3:
16,384 dense x 1 MiB), each on all-0xff virgin maps (reset between steps, as bench.py's
novelty_heavy variant), then STEPS fresh batches on the warm map, with no stage events, so the
trace shows every kernel of both kinds of step as the plain pipeline runs them.  Prints one JSON
line: ms per step by HIP events around each triage.
usage: novelty_trace.py STEPS [dynamorio|afl|afl_classify] [config2|config3]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from killerbeez_amd import synth  # noqa: E402
from killerbeez_amd.triage import MODES, WANT_H32, TriageContext  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = MODES[sys.argv[2]] if len(sys.argv) > 2 else MODES["dynamorio"]
workload = sys.argv[3] if len(sys.argv) > 3 else "config2"  # config3: 16,384 dense x 1 MiB
B, M = (16384, 1 << 20) if workload == "config3" else (65536, 65536)
gen = synth.dense_torch if workload == "config3" else synth.sparse_torch
want = WANT_H32 if mode == MODES["dynamorio"] else 0
dev = torch.device("cuda", 0)
# steps novelty-heavy batches, then steps fresh batches on the warm map (the same trace holds
# both, for attribution: the first `steps` pass-1 dispatches after the warm-up are novelty-heavy)
pool = [gen(B, M, seed=0x5EED + 7919 * p, device=dev, hot_seed=0x5EED)
        for p in range(2 * steps + 1)]
fresh = np.full((3, M), 0xFF, np.uint8)
ms = []
with TriageContext(M, mode, B) as c:
    out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev)}
    if want:
        out["h32"] = torch.empty(B, dtype=torch.int32, device=dev)
    c.triage(*pool[0], want, out=out)
    c.sync()
    for i in range(steps):
        c.set_virgin(fresh)
        c.last_hash = 0
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        c.triage(*pool[i + 1], want, out=out)
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
        c.sync()
    st = c.stats()
    fresh_ms = []
    for i in range(steps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        c.triage(*pool[steps + i + 1], want, out=out)
        b.record()
        b.synchronize()
        fresh_ms.append(a.elapsed_time(b))
        c.sync()
print(json.dumps({"workload": workload, "mode": sys.argv[2] if len(sys.argv) > 2 else "dynamorio",
                  "ms_per_step": round(sum(ms) / len(ms), 4), "ms": [round(x, 4) for x in ms],
                  "fresh_ms_per_step": round(sum(fresh_ms) / len(fresh_ms), 4),
                  "fresh_ms": [round(x, 4) for x in fresh_ms],
                  "last_novelty_batch_work": st}))
