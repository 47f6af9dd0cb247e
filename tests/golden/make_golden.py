#!/usr/bin/env python3
"""Generate tests/golden/*.npz -- known-answer vectors produced by the REFERENCE's own code.

Every expected value below comes from oracle/_ref/libkbz_ref.so, i.e. the reference's
functions compiled from /root/reference (see oracle/Makefile): count_class_lookup,
simplify_lookup/simplify_trace, has_new_bits (AFL and DynamoRIO twins),
has_new_bits_with_ignore, classify_counts, merge_bitmaps, hash32, hash32_with_ignore, XXH64.
The per-exec loops composing them mirror afl_instrumentation.c:231-274 (finish_fuzz_round)
and dynamorio_instrumentation.c:1428-1468 (has_new_coverage).

Inputs are stored in the fixtures (sparse: trace index, byte index, value), so the tests do
not depend on any RNG.  Run from the repository root:  python tests/golden/make_golden.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
M = 65536
HASH_CONST = 0xA5B35705


def P(a):
    return a.ctypes.data_as(C.c_void_p)


def sparse(t):
    j, i = np.nonzero(t)
    return j.astype(np.uint32), i.astype(np.uint32), t[j, i].astype(np.uint8)


def ref_loop(R, mode, traces, outcome, ignore=None, last=0):
    n = traces.shape[0]
    V = np.full((3, M), 0xFF, np.uint8)
    hnb = np.zeros(n, np.uint8)
    h32 = np.zeros(n, np.uint32)
    x64 = np.zeros(n, np.uint64)
    for j in range(n):
        t = traces[j].copy()
        oc = int(outcome[j])
        if mode == oracle.MODE_DYNAMORIO:
            R.ref_dr_classify_counts_64k(P(t))
            h = (R.ref_hash32_with_ignore_ref(P(t), P(ignore), M, HASH_CONST) if ignore is not None
                 else R.ref_hash32_ref(P(t), M, HASH_CONST))
            h32[j] = h
            x64[j] = R.ref_xxh64_ref(P(t), M, 0)
            if h == last:
                continue
            last = h
            hnb[j] = (R.ref_dr_has_new_bits_with_ignore_64k(P(t), P(V[0]), P(ignore))
                      if ignore is not None else R.ref_dr_has_new_bits_64k(P(t), P(V[0])))
        else:
            if oc in (oracle.FUZZ_HANG, oracle.FUZZ_CRASH):
                R.ref_afl_simplify_trace_64k(P(t))
                vm = V[1] if oc == oracle.FUZZ_HANG else V[2]
            else:
                if mode == oracle.MODE_AFL_CLASSIFY:
                    R.ref_dr_classify_counts_64k(P(t))
                vm = V[0]
            h32[j] = R.ref_hash32_ref(P(t), M, HASH_CONST)
            x64[j] = R.ref_xxh64_ref(P(t), M, 0)
            hnb[j] = R.ref_afl_has_new_bits_64k(P(vm), P(t))
    return hnb, h32, x64, V, last


def gen_traces(rng, n, density, hot=None):
    t = np.zeros((n, M), np.uint8)
    for j in range(n):
        k = int(M * density)
        idx = rng.choice(M, size=k, replace=False)
        t[j, idx] = rng.geometric(0.3, size=k).clip(1, 255)
        if hot is not None:
            inc = rng.random(hot.size) < 0.8
            t[j, hot[inc]] = rng.integers(1, 256, size=int(inc.sum()))
    return t


def main():
    oracle.build()
    R = oracle.ref()
    rng = np.random.default_rng(20261015)

    # 1. byte tables
    cc = np.array([R.ref_dr_count_class_64k(c) for c in range(256)], np.uint8)
    simp = np.zeros(256, np.uint8)
    for c in range(256):
        t = np.full(M, c, np.uint8)
        R.ref_afl_simplify_trace_64k(P(t))
        simp[c] = t[0]
    np.savez_compressed(os.path.join(OUT, "tables.npz"), count_class=cc, simplify=simp)

    # 2. hash KATs
    lens = np.array([8, 64, 256, 4096, 65536], np.uint32)
    bufs = [rng.integers(0, 256, size=int(n)).astype(np.uint8) for n in lens]
    for b in bufs:
        b[rng.random(b.size) < 0.7] = 0  # sparse-ish like coverage maps
    ign = [np.where(rng.random(int(n)) < 0.5, 0, 0xFF).astype(np.uint8) for n in lens]
    h32 = np.array([R.ref_hash32_ref(P(b), b.size, HASH_CONST) for b in bufs], np.uint32)
    h32i = np.array([R.ref_hash32_with_ignore_ref(P(b), P(g), b.size, HASH_CONST)
                     for b, g in zip(bufs, ign)], np.uint32)
    xl = np.array([0, 1, 3, 4, 7, 8, 31, 32, 33, 100, 4096, 65536], np.uint32)
    xb = rng.integers(0, 256, size=65536).astype(np.uint8)
    x64 = np.array([R.ref_xxh64_ref(P(xb) if n else None, int(n), 0) for n in xl], np.uint64)
    x64s = np.array([R.ref_xxh64_ref(P(xb) if n else None, int(n), 0x9E3779B97F4A7C15)
                     for n in xl], np.uint64)
    np.savez_compressed(os.path.join(OUT, "hashes.npz"), lens=lens,
                        bufs=np.concatenate(bufs), ignore=np.concatenate(ign), hash32=h32,
                        hash32_ignore=h32i, xxh_lens=xl, xxh_buf=xb, xxh64=x64,
                        xxh64_seeded=x64s)

    # 3. batch triage KATs (three modes), 64 KiB maps
    hot = rng.choice(M, size=200, replace=False)
    n = 80
    t = gen_traces(rng, n, 0.003, hot)
    t[11] = t[10]          # identical neighbours (DynamoRIO last-hash skip)
    t[64] = t[63]          # ... across a 64-trace chunk boundary
    t[70] = 0              # an empty trace
    oc = rng.choice(3, size=n, p=[0.7, 0.15, 0.15]).astype(np.int8)
    oc[10] = oc[11] = oc[63] = oc[64] = 0
    j, i, v = sparse(t)
    fx = dict(n=n, map_size=M, tj=j, ti=i, tv=v, outcome=oc)
    for mode, name in ((oracle.MODE_AFL, "afl"), (oracle.MODE_DYNAMORIO, "dynamorio"),
                       (oracle.MODE_AFL_CLASSIFY, "afl_classify")):
        hnb, hh, xx, V, last = ref_loop(R, mode, t, oc)
        vj, vi = np.nonzero(V != 0xFF)
        fx.update({f"{name}_hnb": hnb, f"{name}_h32": hh, f"{name}_x64": xx,
                   f"{name}_vmap": vj.astype(np.uint8), f"{name}_vidx": vi.astype(np.uint32),
                   f"{name}_vval": V[vj, vi], f"{name}_last": np.uint32(last)})
    # DynamoRIO with ignore_bytes: traces equal under the hash mask, different where
    # has_new_bits_with_ignore looks
    ignb = np.where(rng.random(M) < 0.5, 0, 0xFF).astype(np.uint8)
    t2 = gen_traces(rng, 40, 0.003, hot)
    zc = np.nonzero(ignb == 0)[0]
    for jj in (5, 6, 30):
        t2[jj] = t2[jj - 1]
        t2[jj, rng.choice(zc, 10)] = rng.integers(1, 256, 10)
    oc2 = np.zeros(40, np.int8)
    hnb, hh, xx, V, last = ref_loop(R, oracle.MODE_DYNAMORIO, t2, oc2, ignore=ignb)
    j2, i2, v2 = sparse(t2)
    vj, vi = np.nonzero(V != 0xFF)
    fx.update(dict(ign_n=40, ign_tj=j2, ign_ti=i2, ign_tv=v2, ign_bytes=ignb, ign_hnb=hnb,
                   ign_h32=hh, ign_vmap=vj.astype(np.uint8), ign_vidx=vi.astype(np.uint32),
                   ign_vval=V[vj, vi], ign_last=np.uint32(last)))
    np.savez_compressed(os.path.join(OUT, "triage.npz"), **fx)

    # 4. merger: AND-fold of 5 states (3 virgin maps each), via the reference merge_bitmaps
    states = np.full((5, 3, M), 0xFF, np.uint8)
    for s in range(5):
        for k in range(3):
            idx = rng.choice(M, size=300, replace=False)
            states[s, k, idx] = rng.integers(0, 255, size=300)
    acc = states[0].copy()
    for s in range(1, 5):
        for k in range(3):
            R.ref_afl_merge_bitmaps_64k(P(acc[k]), P(np.ascontiguousarray(states[s, k])))
    sj, sk, si = np.nonzero(states != 0xFF)
    aj, ai = np.nonzero(acc != 0xFF)
    np.savez_compressed(os.path.join(OUT, "merge.npz"), s_state=sj.astype(np.uint8),
                        s_map=sk.astype(np.uint8), s_idx=si.astype(np.uint32),
                        s_val=states[sj, sk, si], m_map=aj.astype(np.uint8),
                        m_idx=ai.astype(np.uint32), m_val=acc[aj, ai])
    picker_fixture(R)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


def picker_fixture(R):
    """5. picker ignore-bytes diff (picker/main.c:240-262), run by the reference's own loop:
    3 files x 5 iterations x 4096 B; per file a sparse base trace, per iteration ~20 noisy
    bytes, iteration 3 of file 1 identical to iteration 2 (a zero pair count)."""
    rng = np.random.default_rng(0x91C4)
    F, I, S = 3, 5, 4096
    runs = np.zeros((F, I, S), np.uint8)
    for f in range(F):
        base = np.zeros(S, np.uint8)
        idx = rng.choice(S, size=200, replace=False)
        base[idx] = rng.integers(1, 256, size=200)
        for it in range(I):
            runs[f, it] = base
            if f == 1 and it == 3:
                runs[f, it] = runs[f, it - 1]
                continue
            noisy = rng.choice(S, size=20, replace=False)
            runs[f, it, noisy] = rng.integers(0, 256, size=20)
    ign = np.empty(S, np.uint8)
    pc = np.zeros((F, I - 1), np.uint32)
    tot = R.ref_picker_ignore_ref(P(runs), F, I, S, P(ign), P(pc))
    rf, ri, rs = np.nonzero(runs)
    np.savez_compressed(os.path.join(OUT, "picker.npz"), shape=np.array([F, I, S], np.uint32),
                        r_file=rf.astype(np.uint8), r_iter=ri.astype(np.uint8),
                        r_idx=rs.astype(np.uint32), r_val=runs[rf, ri, rs],
                        ign_zero=np.nonzero(ign == 0)[0].astype(np.uint32),
                        ign_other=np.array(sorted(set(ign.tolist()) - {0}), np.uint8),
                        pair_counts=pc, total=np.array(tot, np.int64))


if __name__ == "__main__":
    if sys.argv[1:] == ["picker"]:
        oracle.build()
        picker_fixture(oracle.ref())
    else:
        main()
