#!/usr/bin/env python3
"""Diagnostic (not the product): config-2 novelty-heavy steps for a rocprofv3 --kernel-trace run.
A warmed-up DynamoRIO context triages STEPS never-seen 65,536 x 64 KiB batches, each on all-0xff
virgin maps (reset between steps, as bench.py's novelty_heavy variant), with no stage events, so
the trace shows every kernel of those steps as the plain pipeline runs them.  Prints one JSON
line: ms per step by HIP events around each triage."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from killerbeez_amd import synth  # noqa: E402
from killerbeez_amd.triage import MODES, WANT_H32, TriageContext  # noqa: E402

B, M = 65536, 65536
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = MODES[sys.argv[2]] if len(sys.argv) > 2 else MODES["dynamorio"]
want = WANT_H32 if mode == MODES["dynamorio"] else 0
dev = torch.device("cuda", 0)
pool = [synth.sparse_torch(B, M, seed=0x5EED + 7919 * p, device=dev, hot_seed=0x5EED)
        for p in range(steps + 1)]
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
print(json.dumps({"ms_per_step": round(sum(ms) / len(ms), 4), "ms": [round(x, 4) for x in ms],
                  "last_batch_work": st}))
