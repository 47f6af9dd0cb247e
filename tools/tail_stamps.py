#!/usr/bin/env python3
"""k_scan / k_tail per-wave records of a KBZ_TAIL_STAMPS build (diagnostic only, never for results):
config-2 (or KBZ_TAIL_WORKLOAD=config3) fresh batches (bench.py's generator), then, per batch, the distribution of
wave durations in k_scan, the prologue share, and the work of the slowest waves (chunks walked,
inline claims, window items).
usage: KBZ_HIP_LIB=build_variants/tailst/libkbz_hip.so python tools/tail_stamps.py [mode]
(the k_tail path: the fused one-shard tail; per_class splits k_tail's waves by class)"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from killerbeez_amd import _lib, synth  # noqa: E402
from killerbeez_amd.triage import MODES, WANT_H32, TriageContext  # noqa: E402

mode_name = sys.argv[1] if len(sys.argv) > 1 else "dynamorio"
WORKLOAD = os.environ.get("KBZ_TAIL_WORKLOAD", "config2")
B, M = (16384, 1 << 20) if WORKLOAD == "config3" else (65536, 65536)
gen = synth.dense_torch if WORKLOAD == "config3" else synth.sparse_torch
L = _lib.lib()
assert L.kbz_build_flags() != b"", "needs the KBZ_TAIL_STAMPS variant (KBZ_HIP_LIB=...)"
f = L.kbz_debug_tail
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_size_t]
NREC = 1 << 16
NF = 8  # fields per wave record (kTailFields)
FIN_BASE = NREC // 2  # kFinStampBase
buf = np.zeros(NREC * NF, np.uint64)
dev = torch.device("cuda:0")
mode = MODES[mode_name]
want = WANT_H32 if mode == MODES["dynamorio"] else 0
NB = int(os.environ.get("KBZ_TAIL_BATCHES", "8"))  # the bench times batches 4..23
pool = [gen(B, M, seed=1 + 7919 * p, device=dev, hot_seed=1) for p in range(NB)]
out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev)}
res = []
NOVELTY = os.environ.get("KBZ_TAIL_NOVELTY") == "1"  # every batch on all-0xff maps
with TriageContext(M, mode, B) as ctx:
    for i, (t, oc) in enumerate(pool):
        if NOVELTY and i:
            ctx.set_virgin(np.full((3, M), 0xFF, np.uint8))
            ctx.last_hash = 0
            torch.cuda.synchronize()
        f(buf.ctypes.data, 0)  # clears the records
        ctx.triage(t, oc, want, out=out)
        torch.cuda.synchronize()
        ctx.sync()
        assert f(buf.ctypes.data, NREC * NF) == 0
        r = buf.reshape(NREC, NF)
        idx = np.nonzero(r[:, 0])[0]
        fin = r[idx[idx >= FIN_BASE]]  # k_fin's waves (claim items only)
        idx = idx[idx < FIN_BASE]
        live = r[idx]
        ncls = 1 if mode == MODES["dynamorio"] else 3
        cls = idx // ((int(idx.max()) + 1) // ncls)  # k_tail's records are numbered class-major
        t0 = live[:, 0].astype(np.int64)
        t1 = live[:, 1].astype(np.int64)
        t2 = live[:, 2].astype(np.int64)
        cnt = live[:, 3]
        walk = (cnt >> 48) & 0xFFFF
        claims = (cnt >> 32) & 0xFFFF
        win = cnt & 0xFFFF
        ph = live[:, 4:8].astype(np.float64) / 100.0
        base = t0.min()
        dur = (t2 - t0) / 100.0  # us (100 MHz)
        order = np.argsort(-dur)
        st = ctx.stats()
        rec = {
            "batch": i, "waves": int(len(live)), "claim_items": st["claims"],
            "span_us": round((t2.max() - base) / 100.0, 2),
            "start_skew_us": round((t0.max() - base) / 100.0, 2),
            "walking_waves": int((walk > 0).sum()),
            "dur_us_p50_p90_max": [round(float(np.percentile(dur, q)), 2) for q in (50, 90, 100)],
            "prologue_us_p50_max": [round(float(np.percentile((t1 - t0) / 100.0, q)), 2)
                                    for q in (50, 100)],
            "walk_total": int(walk.sum()), "claims_total": int(claims.sum()),
            "windows_total": int(win.sum()),
            "per_class": [{"walk": int(walk[cls == z].sum()), "claims": int(claims[cls == z].sum()),
                           "win": int(win[cls == z].sum()),
                           "dur_us_max": round(float(dur[cls == z].max()), 2) if (cls == z).any() else 0}
                          for z in range(ncls)],
            # k_tail walk phases (us): group loads, per-chunk claims, record scores, flushes
            "phase_us_p50": [round(float(np.percentile(ph[:, p], 50)), 2) for p in range(4)],
            "slowest": [{"dur_us": round(float(dur[j]), 2), "start_us": round((t0[j] - base) / 100.0, 2),
                         "prologue_us": round((t1[j] - t0[j]) / 100.0, 2),
                         "phase_us": [round(float(x), 2) for x in ph[j]],
                         "walk": int(walk[j]), "claims": int(claims[j]), "win": int(win[j]),
                         "cls": int(cls[j])}
                        for j in order[:6]],
        }
        if len(fin):
            fd = (fin[:, 2].astype(np.int64) - fin[:, 0].astype(np.int64)) / 100.0
            fph = fin[:, 4:8].astype(np.float64) / 100.0
            fc = fin[:, 3]
            rec["k_fin"] = {
                "waves": int(len(fin)),
                "span_us": round((int(fin[:, 2].max()) - int(fin[:, 0].min())) / 100.0, 2),
                "dur_us_p50_p90_max": [round(float(np.percentile(fd, q)), 2) for q in (50, 90, 100)],
                "window_items": int((fc & 0xFFFF).sum()),
                "byte_items": int(((fc >> 32) & 0xFFFF).sum()),
                # phase sums per wave (us): windows, byte-item flushes, the rest of the loop,
                # the ticket; p50 / max
                "phase_us_p50": [round(float(np.percentile(fph[:, p], 50)), 2) for p in range(4)],
                "phase_us_max": [round(float(fph[:, p].max()), 2) for p in range(4)],
            }
        res.append(rec)
        print(json.dumps(rec), flush=True)
