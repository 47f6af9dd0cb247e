#!/usr/bin/env python3
"""Does the physical layout of the input batches set pass-1 time?  Same process, same data:
config-2 batches in torch's allocations vs copies in hipExtMallocWithFlags(default) and
hipExtMallocWithFlags(hipDeviceMallocContiguous) buffers, timed interleaved (HIP events on every
pass-1 launch).  Diagnostic only (not part of the product).  usage: alloc_probe.py [K] [ROUNDS]"""
import ctypes as C
import sys

import torch

from killerbeez_amd import synth
from killerbeez_amd.triage import MODES, WANT_H32, TriageContext

hip = C.CDLL("libamdhip64.so")


class Buf:
    """A device buffer from hipExtMallocWithFlags, seen by torch through the array interface."""

    def __init__(self, nbytes, flags):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(nbytes), C.c_uint(flags))
        if rc:
            raise RuntimeError(f"hipExtMallocWithFlags(flags={flags}) rc={rc}")
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (self.ptr, False), "version": 3}

    def free(self):
        hip.hipFree(C.c_void_p(self.ptr))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    B = M = 65536
    base = [synth.sparse_torch(B, M, seed=11 + 7919 * i, device="cuda", hot_seed=11) for i in range(K)]
    kinds = {"torch": base}
    bufs = []
    for name, flags in (("ext_default", 0), ("ext_contiguous", 4)):
        try:
            lst = []
            for t, oc in base:
                b = Buf(B * M, flags)
                bufs.append(b)
                tt = torch.as_tensor(b, device="cuda").view(B, M)
                tt.copy_(t)
                lst.append((tt, oc))
            kinds[name] = lst
        except Exception as e:  # noqa: BLE001
            print(name, "unavailable:", e)
    torch.cuda.synchronize()
    ctx = TriageContext(M, MODES["dynamorio"], B)
    out = {"hnb": torch.empty(B, dtype=torch.uint8, device="cuda"),
           "h32": torch.empty(B, dtype=torch.int32, device="cuda")}
    for t, oc in base[:2]:
        ctx.triage(t, oc, WANT_H32, out=out)
    ctx.sync()
    res = {k: [] for k in kinds}
    for r in range(R):
        for k, lst in kinds.items():
            ctx.sync()
            ctx.time_pass1(True)
            for t, oc in lst:
                ctx.triage(t, oc, WANT_H32, out=out)
            ms, n = ctx.time_pass1(False)
            ctx.sync()
            res[k].append(ms / max(1, n))
    for k, v in res.items():
        print(f"{k:16s} pass1 ms per launch: " + " ".join(f"{x:.4f}" for x in v) +
              f"  mean {sum(v) / len(v):.4f}")
    for b in bufs:
        b.free()


if __name__ == "__main__":
    main()
