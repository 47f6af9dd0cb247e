"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes front-ends for
  * ``libkbz_oracle.so``  -- the clean-room C restatement (oracle/kbz_oracle.c), built on
    CPU here and shipped to the GPU box as the checker / CPU baseline;
  * ``_ref/libkbz_ref.so`` -- the reference's own bitmap code compiled from /root/reference
    by oracle/Makefile (absent where /root/reference is absent).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package.  The product (killerbeez_amd / libkbz_hip.so) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkbz_oracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libkbz_ref.so")

MODE_AFL, MODE_DYNAMORIO, MODE_AFL_CLASSIFY = 0, 1, 2
FUZZ_NONE, FUZZ_HANG, FUZZ_CRASH = 0, 1, 2
WANT_H32, WANT_X64 = 1, 2
HASH_CONST = 0xA5B35705

_u8p = C.POINTER(C.c_uint8)
_lib = None
_ref = None


def build(force: bool = False) -> None:
    """Compile the restatement (and the reference oracle when /root/reference exists)."""
    # make decides what is stale (sources, and the Makefile's flags for the reference build)
    subprocess.check_call(["make", "-s", "-C", HERE, *(["-B"] if force else []), "libkbz_oracle.so"])
    if os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", HERE, *(["-B"] if force else []), "ref"])


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.c_void_p)


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("KBZ_ORACLE_LIB") or LIB_PATH  # scripts/sanitize.sh: ASan build
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.kbzo_count_class.restype = C.c_uint8
        L.kbzo_count_class.argtypes = [C.c_uint8]
        L.kbzo_classify_counts.argtypes = [C.c_void_p, C.c_size_t]
        L.kbzo_simplify_trace.argtypes = [C.c_void_p, C.c_size_t]
        L.kbzo_has_new_bits.restype = C.c_uint8
        L.kbzo_has_new_bits.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.kbzo_has_new_bits_with_ignore.restype = C.c_uint8
        L.kbzo_has_new_bits_with_ignore.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.kbzo_hash32.restype = C.c_uint32
        L.kbzo_hash32.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.kbzo_hash32_with_ignore.restype = C.c_uint32
        L.kbzo_hash32_with_ignore.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]
        L.kbzo_xxh64.restype = C.c_uint64
        L.kbzo_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.kbzo_merge_and.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.kbzo_merge_many.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t]
        L.kbzo_ipt_keys.restype = C.c_size_t
        L.kbzo_ipt_keys.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
        L.kbzo_picker_ignore.restype = C.c_size_t
        L.kbzo_picker_ignore.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                         C.c_void_p, C.c_void_p]
        args = [C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p,
                C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                C.c_void_p]
        L.kbzo_triage_batch.restype = C.c_int
        L.kbzo_triage_batch.argtypes = args
        L.kbzo_triage_batch_mt.restype = C.c_int
        L.kbzo_triage_batch_mt.argtypes = args + [C.c_int]
        L.kbzo_cpu_probe.restype = C.c_double
        L.kbzo_cpu_probe.argtypes = [C.c_int, C.c_long]
        L.kbzo_mem_probe.restype = C.c_double
        L.kbzo_mem_probe.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_int]
        _lib = L
    return _lib


def cpu_cores_granted(threads: int, iters: int = 200_000_000) -> float:
    """Cores this process actually gets with `threads` OpenMP threads: one register-only
    chain per thread, threads x t(1) / t(threads)."""
    t1 = lib().kbzo_cpu_probe(1, iters)
    tn = lib().kbzo_cpu_probe(threads, iters)
    return threads * t1 / tn if tn > 0 else 0.0


def have_ref() -> bool:
    return os.path.exists(REF_PATH)


def ref():
    """The reference's own code (oracle/_ref).  Raises if it was not built."""
    global _ref
    if _ref is None:
        if not have_ref():
            raise FileNotFoundError(REF_PATH)
        R = C.CDLL(REF_PATH)
        for sfx in ("64k", "1m"):
            f = getattr(R, f"ref_afl_has_new_bits_{sfx}")
            f.restype, f.argtypes = C.c_uint8, [C.c_void_p, C.c_void_p]
            getattr(R, f"ref_afl_simplify_trace_{sfx}").argtypes = [C.c_void_p]
            getattr(R, f"ref_afl_merge_bitmaps_{sfx}").argtypes = [C.c_void_p, C.c_void_p]
            f = getattr(R, f"ref_dr_has_new_bits_{sfx}")
            f.restype, f.argtypes = C.c_uint8, [C.c_void_p, C.c_void_p]
            f = getattr(R, f"ref_dr_has_new_bits_with_ignore_{sfx}")
            f.restype, f.argtypes = C.c_uint8, [C.c_void_p, C.c_void_p, C.c_void_p]
            getattr(R, f"ref_dr_classify_counts_{sfx}").argtypes = [C.c_void_p]
            getattr(R, f"ref_dr_merge_bitmaps_{sfx}").argtypes = [C.c_void_p, C.c_void_p]
            f = getattr(R, f"ref_dr_count_class_{sfx}")
            f.restype, f.argtypes = C.c_uint8, [C.c_uint8]
        R.ref_hash32_ref.restype = C.c_uint32
        R.ref_hash32_ref.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        R.ref_winafl_hash32_ref.restype = C.c_uint32
        R.ref_winafl_hash32_ref.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        R.ref_hash32_with_ignore_ref.restype = C.c_uint32
        R.ref_hash32_with_ignore_ref.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]
        R.ref_xxh64_ref.restype = C.c_uint64
        R.ref_xxh64_ref.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        R.ref_xxh_version_ref.restype = C.c_uint
        R.ref_ipt_keys_ref.restype = C.c_size_t
        R.ref_ipt_keys_ref.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
        R.ref_picker_ignore_ref.restype = C.c_int
        R.ref_picker_ignore_ref.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p]
        _ref = R
    return _ref


# ---- numpy conveniences over the restatement ------------------------------------------------

def count_class_table() -> np.ndarray:
    L = lib()
    return np.array([L.kbzo_count_class(c) for c in range(256)], dtype=np.uint8)


def hash32(buf: np.ndarray, seed: int = HASH_CONST) -> int:
    b = np.ascontiguousarray(buf, dtype=np.uint8)
    return int(lib().kbzo_hash32(_p(b), b.size, seed))


def xxh64(buf: np.ndarray, seed: int = 0) -> int:
    b = np.ascontiguousarray(buf, dtype=np.uint8)
    return int(lib().kbzo_xxh64(_p(b), b.size, seed))


def triage_batch(mode, traces, outcome=None, virgin=None, ignore=None, last_hash=0,
                 want=WANT_H32, threads=0):
    """Sequential (threads==0) or sharded (threads>=1) CPU triage.

    traces: uint8 [n, map_size].  virgin: uint8 [3, map_size] (modified copy returned).
    Returns dict(hnb, h32, x64, virgin, last_hash)."""
    t = np.ascontiguousarray(traces, dtype=np.uint8)
    n, m = t.shape
    v = np.full((3, m), 0xFF, np.uint8) if virgin is None else np.array(virgin, np.uint8, copy=True)
    oc = None if outcome is None else np.ascontiguousarray(outcome, dtype=np.int8)
    ig = None if ignore is None else np.ascontiguousarray(ignore, dtype=np.uint8)
    hnb = np.zeros(n, np.uint8)
    h32 = np.zeros(n, np.uint32)
    x64 = np.zeros(n, np.uint64)
    lh = C.c_uint32(last_hash)
    a = (mode, _p(t), n, m, m, _p(oc), _p(v), _p(ig), C.byref(lh), want, _p(hnb), _p(h32),
         _p(x64))
    rc = lib().kbzo_triage_batch(*a) if threads == 0 else lib().kbzo_triage_batch_mt(*a, threads)
    if rc:
        raise ValueError("kbzo_triage_batch: bad arguments")
    return dict(hnb=hnb, h32=h32, x64=x64, virgin=v, last_hash=lh.value)


def transform(traces: np.ndarray, xf: int) -> np.ndarray:
    """classify_counts (xf=1, dynamorio_instrumentation.c:265-292) or simplify_trace (xf=2,
    afl_instrumentation.c:674-706) of every row (restated; returns a transformed copy)."""
    t = np.array(traces, np.uint8, copy=True)
    if xf == 0:
        return t
    f = lib().kbzo_classify_counts if xf == 1 else lib().kbzo_simplify_trace
    flat = t.reshape(-1, t.shape[-1])
    for row in flat:
        f(_p(row), row.size)
    return t


def merge_many(states: np.ndarray) -> np.ndarray:
    s = np.ascontiguousarray(states, dtype=np.uint8)
    n = s.shape[0]
    per = s[0].size if n else 0
    out = np.empty(per, np.uint8)
    lib().kbzo_merge_many(_p(out), _p(s), n, per)
    return out.reshape(s.shape[1:])


def picker_ignore(runs: np.ndarray):
    """Restated picker diff (picker/main.c:240-262) over runs [files, iters, size]:
    (ignore [size], pair_counts [files, iters-1] uint32, total)."""
    r = np.ascontiguousarray(runs, dtype=np.uint8)
    files, iters, size = r.shape
    ign = np.empty(size, np.uint8)
    pc = np.zeros((files, max(iters - 1, 0)), np.uint32)
    tot = lib().kbzo_picker_ignore(_p(r), files, iters, size, _p(ign), _p(pc) if pc.size else None)
    return ign, pc, int(tot)


def ipt_keys(events: np.ndarray, lib_starts=(), lib_ends=(), lib_hashes=(), target_start=0,
             target_end=0, use_ref: bool = False) -> np.ndarray:
    """Intel-PT path keys [execs, 2] = {tip, tnt} from events uint64 [k, 3] (kind, a, b): the
    restatement, or the reference's own feeders (oracle/_ref) with use_ref."""
    ev = np.ascontiguousarray(events, dtype=np.uint64).reshape(-1, 3)
    ls = np.ascontiguousarray(lib_starts, dtype=np.uint64)
    le = np.ascontiguousarray(lib_ends, dtype=np.uint64)
    lh = np.ascontiguousarray(lib_hashes, dtype=np.uint32)
    out = np.zeros((max(1, int((ev[:, 0] == 2).sum())), 2), np.uint64)
    f = ref().ref_ipt_keys_ref if use_ref else lib().kbzo_ipt_keys
    n = f(_p(ev), ev.shape[0], ls.size, _p(ls), _p(le), _p(lh), int(target_start),
          int(target_end), _p(out))
    return out[:n]


def host_read_gbps(threads: int, buf: np.ndarray, passes: int = 3) -> float:
    """Host memory read bandwidth (GB/s) of `threads` threads streaming disjoint slices of buf."""
    b = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    el = lib().kbzo_mem_probe(threads, _p(b), b.size, passes)
    return passes * b.size / el / 1e9 if el > 0 else 0.0
