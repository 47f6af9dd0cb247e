#!/usr/bin/env python3
"""Diagnostic: run pass 1 of the bench workload with a -DKBZ_STAMPS build of libkbz_hip.so and
print the per-wave cycle split of each step {compute, vmcnt wait, fill+prefetch, barrier}
for wave L (loader/chain) and wave T (transform).  Not part of the product."""
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
t, oc = synth.sparse_torch(65536, 65536, device="cuda")
ctx = TriageContext(65536, 1, 65536)
for _ in range(3):
    ctx.triage(t, oc, WANT_H32)
torch.cuda.synchronize()
buf = np.zeros(4096 * 2 * 4, np.uint64)
f(buf.ctypes.data_as(C.c_void_p), buf.size)
st = buf.reshape(4096, 2, 4)[:1024].astype(np.float64)
names = ["compute", "vmcnt wait", "fill+prefetch", "barrier"]
for w, wn in ((0, "L"), (1, "T")):
    tot = st[:, w, :].sum(axis=1)
    print(f"wave {wn}: total cycles/wave median {np.median(tot):.0f}")
    for i, n in enumerate(names):
        print(f"   {n:14s} {np.median(st[:, w, i]):10.0f}  ({100*np.median(st[:, w, i]/tot):.1f}%)")
