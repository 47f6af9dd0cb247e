#!/usr/bin/env python3
"""Diagnostic: run the wide DynamoRIO pass 1 on BASELINE config 3 (16,384 dense x 1 MiB) with a
-DKBZ_STAMPS build (KBZ_HIP_LIB=...) and print, per wave of the workgroup, the median cycles per
launch in its four stamp phases.  k_pass1w: {work, barrier wait, vmcnt wait / finish, LDS fill};
k_pass1d (KBZ_STAMP_NAMES=d): C wave 0 {chain, ready wait, LDS read wait, flags}, X waves
{vmcnt wait, classify+OR+mix, freed wait, ring writes+stores+loads}.  Not part of the product."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from killerbeez_amd import synth  # noqa: E402
from killerbeez_amd._lib import lib  # noqa: E402
from killerbeez_amd.triage import WANT_H32, TriageContext  # noqa: E402

L = lib()
f = L.kbz_debug_stamps
f.argtypes = [C.c_void_p, C.c_size_t]
n, M = 16384, 1 << 20
t, oc = synth.dense_torch(n, M, device="cuda")
ctx = TriageContext(M, 1, n)
for _ in range(3):
    ctx.triage(t, oc, WANT_H32)
torch.cuda.synchronize()
buf = np.zeros(4096 * 2 * 4, np.uint64)
f(buf.ctypes.data_as(C.c_void_p), buf.size)
st = buf.reshape(-1, 16, 4)[:256].astype(np.float64)  # [chunk][wave][phase]
D_NAMES = {"C": ["chain", "ready wait", "LDS read wait", "flag read"],
           "N": ["compare", "ready wait", "LDS read wait", "-"],
           "X": ["vmcnt wait", "classify+OR", "freed wait", "mix+ring+stores+loads"]}
dmode = os.environ.get("KBZ_STAMP_NAMES") == "d"
for w in range(16):
    tot = st[:, w, :].sum(axis=1)
    if np.median(tot) == 0:
        continue
    if dmode:
        kind = "C" if w == 0 else "N" if w == 4 else "X"
        names = D_NAMES[kind]
    else:
        kind, names = "", ["work|xform", "barrier", "vmcnt|reads", "fill|finish"]
    cols = "  ".join(f"{nm} {np.median(st[:, w, i]) / 1e6:7.3f}M ({100 * np.median(st[:, w, i] / tot):4.1f}%)"
                     for i, nm in enumerate(names))
    print(f"wave {w:2d} {kind}: total {np.median(tot) / 1e6:7.3f}M cycles  {cols}")
