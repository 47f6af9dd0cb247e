"""Pin the clean-room restatement (oracle/kbz_oracle.c) to the reference's own code.

oracle/_ref/libkbz_ref.so is compiled from the files under /root/reference by oracle/Makefile
(no reference source is copied into the repo).  Every restated function is compared with the
reference function it restates on seeded random inputs, both map sizes.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from killerbeez_amd import synth

pytestmark = pytest.mark.skipif(not oracle.have_ref() and not __import__("os").path.isdir(
    "/root/reference"), reason="reference oracle not available")


@pytest.fixture(scope="module")
def R(oracle_lib):
    oracle.build()
    if not oracle.have_ref():
        pytest.skip("oracle/_ref not built")
    return oracle.ref()


def P(a):
    return a.ctypes.data_as(C.c_void_p)


SFX = {65536: "64k", 1 << 20: "1m"}


def rand_trace(rng, m, density):
    t = np.zeros(m, np.uint8)
    k = int(m * density)
    idx = rng.choice(m, size=k, replace=False)
    t[idx] = rng.integers(1, 256, size=k)
    return t


def test_xxhash_version(R):
    assert R.ref_xxh_version_ref() == 605  # vendored xxHash v0.6.5 (xxhash.h:155-158)


def test_count_class_exhaustive(R):
    L = oracle.lib()
    for c in range(256):
        assert L.kbzo_count_class(c) == R.ref_dr_count_class_64k(c)


@pytest.mark.parametrize("m", [65536, 1 << 20])
def test_transforms_and_has_new_bits(R, m):
    rng = np.random.default_rng(1)
    L = oracle.lib()
    sfx = SFX[m]
    for density in (0.0, 0.001, 0.02, 0.5, 1.0):
        t = rand_trace(rng, m, density)
        a, b = t.copy(), t.copy()
        getattr(R, f"ref_dr_classify_counts_{sfx}")(P(a))
        L.kbzo_classify_counts(P(b), m)
        assert np.array_equal(a, b)
        a, b = t.copy(), t.copy()
        getattr(R, f"ref_afl_simplify_trace_{sfx}")(P(a))
        L.kbzo_simplify_trace(P(b), m)
        assert np.array_equal(a, b)
    # has_new_bits (AFL and DR variants) on a running sequence
    va = np.full(m, 0xFF, np.uint8)
    vd, vo = va.copy(), va.copy()
    for k in range(12):
        t = rand_trace(rng, m, [0.001, 0.02, 0.3][k % 3])
        ra = getattr(R, f"ref_afl_has_new_bits_{sfx}")(P(va), P(t))
        rd = getattr(R, f"ref_dr_has_new_bits_{sfx}")(P(t), P(vd))
        ro = L.kbzo_has_new_bits(P(vo), P(t), m)
        assert ra == rd == ro
        assert np.array_equal(va, vo) and np.array_equal(vd, vo)


def test_has_new_bits_with_ignore(R):
    m = 65536
    rng = np.random.default_rng(2)
    L = oracle.lib()
    ign = np.where(rng.random(m) < 0.3, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
    v1 = np.full(m, 0xFF, np.uint8)
    v2 = v1.copy()
    for k in range(10):
        t = rand_trace(rng, m, 0.05)
        r1 = R.ref_dr_has_new_bits_with_ignore_64k(P(t), P(v1), P(ign))
        r2 = L.kbzo_has_new_bits_with_ignore(P(t), P(v2), P(ign), m)
        assert r1 == r2 and np.array_equal(v1, v2)


def test_hashes(R):
    import xxhash

    rng = np.random.default_rng(3)
    L = oracle.lib()
    for m in (8, 64, 4096, 65536, 1 << 20):
        for density in (0.0, 0.02, 1.0):
            t = rand_trace(rng, m, density)
            ig = rng.integers(0, 256, size=m).astype(np.uint8)
            assert R.ref_hash32_ref(P(t), m, oracle.HASH_CONST) == L.kbzo_hash32(P(t), m, oracle.HASH_CONST)
            assert R.ref_winafl_hash32_ref(P(t), m, 7) == L.kbzo_hash32(P(t), m, 7)
            assert (R.ref_hash32_with_ignore_ref(P(t), P(ig), m, oracle.HASH_CONST)
                    == L.kbzo_hash32_with_ignore(P(t), P(ig), m, oracle.HASH_CONST))
    for ln in (0, 1, 3, 4, 7, 8, 31, 32, 33, 63, 100, 4096, 65536):
        t = rng.integers(0, 256, size=max(ln, 1)).astype(np.uint8)[:ln]
        for seed in (0, 1, 0xA5B35705):
            r = R.ref_xxh64_ref(P(t) if ln else None, ln, seed)
            assert r == L.kbzo_xxh64(P(t) if ln else None, ln, seed)
            assert r == xxhash.xxh64_intdigest(t.tobytes(), seed)


def test_merge(R):
    rng = np.random.default_rng(4)
    L = oracle.lib()
    for m, sfx in ((65536, "64k"), (1 << 20, "1m")):
        a = rng.integers(0, 256, size=m).astype(np.uint8)
        b = rng.integers(0, 256, size=m).astype(np.uint8)
        x, y = a.copy(), a.copy()
        getattr(R, f"ref_afl_merge_bitmaps_{sfx}")(P(x), P(b))
        L.kbzo_merge_and(P(y), P(b), m)
        assert np.array_equal(x, y)
        x = a.copy()
        getattr(R, f"ref_dr_merge_bitmaps_{sfx}")(P(x), P(b))
        assert np.array_equal(x, y)


def ref_triage(R, mode, traces, outcome, ignore=None, last=0):
    """Per-exec loop composed from the reference's own functions, mirroring
    afl_instrumentation.c:231-274 (AFL) and dynamorio_instrumentation.c:1428-1468 (DR)."""
    n, m = traces.shape
    sfx = SFX[m]
    V = np.full((3, m), 0xFF, np.uint8)
    hnb = np.zeros(n, np.uint8)
    for j in range(n):
        t = traces[j].copy()
        oc = int(outcome[j])
        if mode == oracle.MODE_DYNAMORIO:
            getattr(R, f"ref_dr_classify_counts_{sfx}")(P(t))
            h = (R.ref_hash32_with_ignore_ref(P(t), P(ignore), m, oracle.HASH_CONST)
                 if ignore is not None else R.ref_hash32_ref(P(t), m, oracle.HASH_CONST))
            if h == last:
                hnb[j] = 0
                continue
            last = h
            if ignore is not None:
                hnb[j] = getattr(R, f"ref_dr_has_new_bits_with_ignore_{sfx}")(P(t), P(V[0]), P(ignore))
            else:
                hnb[j] = getattr(R, f"ref_dr_has_new_bits_{sfx}")(P(t), P(V[0]))
        else:
            if oc in (oracle.FUZZ_HANG, oracle.FUZZ_CRASH):
                getattr(R, f"ref_afl_simplify_trace_{sfx}")(P(t))
                vm = V[1] if oc == oracle.FUZZ_HANG else V[2]
            else:
                if mode == oracle.MODE_AFL_CLASSIFY:
                    getattr(R, f"ref_dr_classify_counts_{sfx}")(P(t))
                vm = V[0]
            hnb[j] = getattr(R, f"ref_afl_has_new_bits_{sfx}")(P(vm), P(t))
    return hnb, V, last


@pytest.mark.parametrize("mode", [oracle.MODE_AFL, oracle.MODE_DYNAMORIO, oracle.MODE_AFL_CLASSIFY])
def test_batch_triage_matches_reference_loop(R, mode):
    t, oc = synth.sparse_np(160, 65536, seed=11 + mode)
    t[40] = t[39]  # identical neighbours (DynamoRIO last-hash skip)
    t[64] = t[63]
    oc[63] = oc[64] = 0
    hnb, V, last = ref_triage(R, mode, t, oc)
    for threads in (0, 1, 3, 8):
        r = oracle.triage_batch(mode, t, oc, threads=threads)
        assert np.array_equal(r["hnb"], hnb), threads
        assert np.array_equal(r["virgin"][0], V[0])
        if mode != oracle.MODE_DYNAMORIO:
            assert np.array_equal(r["virgin"], V)
        else:
            assert r["last_hash"] == last
    assert hnb.max() == 2 and (hnb == 0).any()


def test_batch_triage_dynamorio_ignore(R):
    rng = np.random.default_rng(9)
    m = 65536
    t, oc = synth.sparse_np(128, m, seed=5)
    ign = np.where(rng.random(m) < 0.5, 0, 0xFF).astype(np.uint8)
    # traces that differ only in bytes the hash masks out (ignore==0) hash equal but differ in
    # the bytes has_new_bits_with_ignore examines
    zero_cols = np.nonzero(ign == 0)[0][:50]
    t[21] = t[20]
    t[21, zero_cols] = 7
    hnb, V, last = ref_triage(R, oracle.MODE_DYNAMORIO, t, oc, ignore=ign)
    for threads in (0, 4):
        r = oracle.triage_batch(oracle.MODE_DYNAMORIO, t, oc, ignore=ign, threads=threads)
        assert np.array_equal(r["hnb"], hnb)
        assert np.array_equal(r["virgin"][0], V[0])
        assert r["last_hash"] == last


@pytest.mark.parametrize("files,iters,size", [(4, 6, 65536), (2, 1, 4096), (0, 3, 256),
                                              (1, 2, 1 << 20)])
def test_picker_ignore(R, files, iters, size):
    """Restated picker diff vs the reference's own loop (picker/main.c:240-262)."""
    rng = np.random.default_rng(files * 100 + iters)
    base = rng.integers(0, 256, size=(files, 1, size), dtype=np.uint8)
    runs = np.repeat(base, iters, axis=1)
    noise = rng.random((files, iters, size)) < 0.01
    runs[noise] = rng.integers(0, 256, size=int(noise.sum()), dtype=np.uint8)
    ign, pc, tot = oracle.picker_ignore(runs)
    r_ign = np.empty(size, np.uint8)
    r_pc = np.zeros((files, max(iters - 1, 0)), np.uint32)
    r_tot = R.ref_picker_ignore_ref(P(runs), files, iters, size, P(r_ign),
                                    P(r_pc) if r_pc.size else None)
    np.testing.assert_array_equal(ign, r_ign)
    np.testing.assert_array_equal(pc, r_pc)
    assert tot == r_tot
