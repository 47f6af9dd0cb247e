"""Bit-exact parity of the gfx950 path (libkbz_hip.so through the C ABI) with the CPU oracle.

The oracle (oracle/kbz_oracle.c) is itself pinned to the reference's own code by
tests/test_oracle_pin.py and to tests/golden/ by tests/test_golden.py.  Every comparison here
is exact: per-trace has_new_bits results, hash32, XXH64, the three virgin maps and the
DynamoRIO last hash.
"""
import numpy as np
import pytest

import oracle
from killerbeez_amd import synth
from killerbeez_amd.triage import (MODE_AFL, MODE_AFL_CLASSIFY, MODE_DYNAMORIO, WANT_H32,
                                   WANT_X64, TriageContext, hash32_rows, merge_and,
                                   merge_and_host, xxh64_rows)

pytestmark = pytest.mark.gpu
MODES = [MODE_AFL, MODE_DYNAMORIO, MODE_AFL_CLASSIFY]


@pytest.fixture(autouse=True, params=["narrow", "wide", "narrow-staged"])
def pass1(request, monkeypatch):
    """Every case runs through both pass-1 kernels: k_pass1s (narrow; what AUTO picks for
    batches of >= 512 chunks, e.g. config 2) and k_pass1w (wide; AUTO's pick below that), and
    through both tails after pass 1: the fused one-shard tail (k_skip + k_tail, what
    kbz_triage_batch_device runs) and the staged kernels the sharded protocol runs (k_skip,
    k_chain, k_total, k_scan, k_resolve, k_pack; KBZ_DEBUG_STAGED=1).  kbz_ctx_create reads
    KBZ_PASS1 / KBZ_DEBUG_STAGED as the new context's defaults."""
    kind = request.param.split("-")[0]
    monkeypatch.setenv("KBZ_PASS1", kind)
    if request.param.endswith("staged"):
        monkeypatch.setenv("KBZ_DEBUG_STAGED", "1")
    return kind


def gpu_triage(ctx, traces, oc, want=WANT_H32 | WANT_X64):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(traces)).cuda()
    o = None if oc is None else torch.from_numpy(np.ascontiguousarray(oc)).cuda()
    out = ctx.triage(t, o, want)
    torch.cuda.synchronize()
    ctx.sync()
    res = {"hnb": out["hnb"].cpu().numpy()}
    if "h32" in out:
        res["h32"] = out["h32"].cpu().numpy().view(np.uint32)
    if "x64" in out:
        res["x64"] = out["x64"].cpu().numpy().view(np.uint64)
    return res


def check(mode, traces, oc, ignore=None, virgin=None, last=0, want=WANT_H32 | WANT_X64,
          ctx=None, max_batch=None):
    n, m = traces.shape
    own = ctx is None
    if own:
        ctx = TriageContext(m, mode, max_batch or max(n, 1))
        if ignore is not None:
            ctx.set_ignore(ignore)
        if virgin is not None:
            ctx.set_virgin(virgin)
        ctx.last_hash = last
    v0 = ctx.get_virgin()
    l0 = ctx.last_hash
    exp = oracle.triage_batch(mode, traces, oc, virgin=v0, ignore=ignore, last_hash=l0,
                              want=oracle.WANT_H32 | oracle.WANT_X64)
    got = gpu_triage(ctx, traces, oc, want)
    np.testing.assert_array_equal(got["hnb"], exp["hnb"])
    if want & WANT_H32:
        np.testing.assert_array_equal(got["h32"], exp["h32"])
    if want & WANT_X64:
        np.testing.assert_array_equal(got["x64"], exp["x64"])
    np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])
    if mode == MODE_DYNAMORIO:
        assert ctx.last_hash == exp["last_hash"]
    if own:
        ctx.close()
    return exp


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_sparse_64k_partial_chunk(gpu, mode, want):
    t, oc = synth.sparse_np(1000, 65536, seed=100 + mode)
    exp = check(mode, t, oc, want=want)
    assert exp["hnb"].max() == 2


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("density", [0.02, 0.3, 1.0])
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_uniform_density(gpu, mode, density, want):
    t = synth.uniform_np(200, 65536, seed=int(density * 100), density=density)
    rng = np.random.default_rng(7)
    oc = rng.choice(3, size=200, p=[0.7, 0.15, 0.15]).astype(np.int8)
    check(mode, t, oc, want=want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("m", [256, 4096, 1 << 20])
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_map_sizes(gpu, mode, m, want):
    t, oc = synth.sparse_np(130, m, seed=m + mode, hot_frac=0.05)
    check(mode, t, oc, want=want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65])
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_small_batches(gpu, mode, n, want):
    t, oc = synth.sparse_np(n, 4096, seed=n)
    check(mode, t, oc, want=want)


def test_dynamorio_identical_runs_and_chunk_boundary(gpu):
    t, oc = synth.sparse_np(300, 65536, seed=3)
    t[10:20] = t[9]        # a run inside a chunk
    t[64] = t[63]          # across the chunk boundary
    t[128:140] = t[127]    # run that starts a chunk
    t[200] = t[198]        # equal to a non-neighbour: not skipped
    exp = check(MODE_DYNAMORIO, t, oc)
    assert (exp["hnb"][10:20] == 0).all() and exp["hnb"][64] == 0


def test_dynamorio_last_hash_carried_across_batches(gpu):
    t, oc = synth.sparse_np(200, 65536, seed=4)
    ctx = TriageContext(65536, MODE_DYNAMORIO, 200)
    check(MODE_DYNAMORIO, t[:100], oc[:100], ctx=ctx)
    t2 = t[100:].copy()
    t2[0] = t[99]  # first trace of batch 2 equals the last of batch 1 -> skipped
    t2[64] = t2[63]
    exp = check(MODE_DYNAMORIO, t2, oc[100:], ctx=ctx)
    assert exp["hnb"][0] == 0
    ctx.close()


def test_dynamorio_ignore_skips_that_differ(gpu):
    """hash32_with_ignore masks bytes whose ignore byte is 0, has_new_bits_with_ignore only
    looks at those bytes: equal hashes with different examined bytes must be excluded from
    the virgin update (the chunk-recompute path)."""
    rng = np.random.default_rng(5)
    m = 65536
    t, oc = synth.sparse_np(400, m, seed=6)
    ign = np.where(rng.random(m) < 0.4, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
    zc = np.nonzero(ign == 0)[0]
    for j in (5, 64, 65, 130, 131, 132, 399):
        t[j] = t[j - 1]
        t[j, rng.choice(zc, 20)] = rng.integers(1, 256, 20)
    check(MODE_DYNAMORIO, t, oc, ignore=ign)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_preset_virgin_and_sequential_composition(gpu, mode, want):
    m = 65536
    rng = np.random.default_rng(8)
    v = rng.integers(0, 256, size=(3, m)).astype(np.uint8)
    v[:, rng.random(m) < 0.5] = 0xFF
    t, oc = synth.sparse_np(700, m, seed=9)
    ctx = TriageContext(m, mode, 700)
    ctx.set_virgin(v)
    # three uneven batches in a row == one sequential pass
    for lo, hi in ((0, 1), (1, 333), (333, 700)):
        check(mode, t[lo:hi], oc[lo:hi], ctx=ctx, want=want)
    whole = oracle.triage_batch(mode, t, oc, virgin=v)
    np.testing.assert_array_equal(ctx.get_virgin(), whole["virgin"])
    ctx.close()


@pytest.mark.parametrize("mode", [MODE_AFL, MODE_AFL_CLASSIFY])
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_crash_hang_heavy(gpu, mode, want):
    t, oc = synth.sparse_np(500, 65536, seed=12, outcome_p=(0.4, 0.3, 0.3))
    check(mode, t, oc, want=want)


@pytest.mark.parametrize("mode", [MODE_AFL, MODE_AFL_CLASSIFY])
@pytest.mark.parametrize("oc_all", [1, 2])
def test_all_hang_or_crash_no_hash(gpu, mode, oc_all):
    """Every exec a hang (or crash): only the simplified class is present (simplify_trace
    afl_instrumentation.c:674-706), with all-zero rows (0x01 everywhere) in some chunks."""
    t, _ = synth.sparse_np(700, 4096, seed=20 + oc_all, hot_frac=0.05)
    t[64:70] = 0
    t[300:364] = 0
    check(mode, t, np.full(700, oc_all, np.int8), want=0)


@pytest.mark.parametrize("mode", MODES)
def test_strided_rows_and_no_outcome(gpu, mode):
    import torch

    m = 4096
    t, oc = synth.sparse_np(150, m, seed=13)
    big = np.zeros((150, m + 512), np.uint8)
    big[:, :m] = t
    ctx = TriageContext(m, mode, 150)
    exp = oracle.triage_batch(mode, t, None, want=oracle.WANT_H32 | oracle.WANT_X64)
    tt = torch.from_numpy(big).cuda()[:, :m]
    out = ctx.triage(tt, None, WANT_H32 | WANT_X64)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
    np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), exp["h32"])
    np.testing.assert_array_equal(out["x64"].cpu().numpy().view(np.uint64), exp["x64"])
    np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])


@pytest.mark.parametrize("mode", MODES)
def test_host_streaming_path(gpu, mode):
    m = 65536
    t, oc = synth.sparse_np(2500, m, seed=14)
    ctx = TriageContext(m, mode, 2500)
    exp = oracle.triage_batch(mode, t, oc, want=oracle.WANT_H32 | oracle.WANT_X64)
    got = ctx.triage_host(t, oc, WANT_H32 | WANT_X64)
    np.testing.assert_array_equal(got["hnb"], exp["hnb"])
    np.testing.assert_array_equal(got["h32"], exp["h32"])
    np.testing.assert_array_equal(got["x64"], exp["x64"])
    np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])


@pytest.mark.parametrize("n,nbytes", [(0, 3 * 4096), (1, 3 * 4096), (37, 3 * 65536),
                                      (1000, 3 * 65536), (20, 1000)])
def test_merge(gpu, n, nbytes):
    import torch

    rng = np.random.default_rng(n)
    s = rng.integers(0, 256, size=(n, nbytes)).astype(np.uint8) | rng.integers(
        0, 256, size=(n, nbytes)).astype(np.uint8)
    exp = oracle.merge_many(s) if n else np.full(nbytes, 0xFF, np.uint8)
    got = merge_and(torch.from_numpy(s).cuda().reshape(n, nbytes)) if n else None
    if got is not None:
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), exp.reshape(-1))
    if n:
        np.testing.assert_array_equal(merge_and_host(s.reshape(n, nbytes)), exp.reshape(-1))


def test_merge_states_property(gpu):
    import torch

    s = synth.merger_states_np(257, 4096, seed=1)
    got = merge_and(torch.from_numpy(s).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, np.bitwise_and.reduce(s, axis=0))


@pytest.mark.parametrize("n,nbytes", [(5000, 4096), (3000, 3 * 65536)])
def test_merge_tree_sparse_clears(gpu, n, nbytes):
    """Enough states for the multi-stage fold tree (5000 x 4 KiB: 312 -> 20 -> 2 partial rows);
    about nbytes*8 bits cleared over all states, so the AND keeps ~1/3 of its bits set."""
    import torch

    rng = np.random.default_rng(n)
    s = np.full((n, nbytes), 0xFF, np.uint8)
    pos = rng.integers(0, n * nbytes * 8, size=nbytes * 8)
    np.bitwise_and.at(s.reshape(-1), pos // 8, ~(np.uint8(1) << (pos % 8).astype(np.uint8)))
    exp = np.bitwise_and.reduce(s, axis=0)
    assert 0.2 < np.unpackbits(exp).mean() < 0.6
    got = merge_and(torch.from_numpy(s).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("length", [8, 64, 256, 4096, 65536])
def test_row_hashes(gpu, length):
    import torch

    rng = np.random.default_rng(length)
    rows = rng.integers(0, 256, size=(70, length)).astype(np.uint8)
    h = hash32_rows(torch.from_numpy(rows).cuda()).cpu().numpy().view(np.uint32)
    x = xxh64_rows(torch.from_numpy(rows).cuda()).cpu().numpy().view(np.uint64)
    for j in range(70):
        assert h[j] == oracle.hash32(rows[j])
        assert x[j] == oracle.xxh64(rows[j])
    for ln in (1, 5, 31, 33, 100):
        x = xxh64_rows(torch.from_numpy(rows).cuda(), length=min(ln, length), seed=3).cpu().numpy().view(np.uint64)
        assert x[0] == oracle.xxh64(rows[0, :min(ln, length)], 3)


@pytest.mark.slow
def test_full_size_config2(gpu):
    """BASELINE config 2 at full size: 65,536 sparse traces x 64 KiB, DynamoRIO mode, checked
    exactly against the sharded CPU oracle, plus size-independent invariants."""
    import torch

    n, m = 65536, 65536
    t, oc = synth.sparse_torch(n, m, seed=0x5EED, device="cuda")
    ctx = TriageContext(m, MODE_DYNAMORIO, n)
    out = ctx.triage(t, oc, WANT_H32)
    torch.cuda.synchronize()
    ctx.sync()
    th = t.cpu().numpy()
    exp = oracle.triage_batch(MODE_DYNAMORIO, th, oc.cpu().numpy(), threads=16)
    np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
    np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), exp["h32"])
    v = ctx.get_virgin()
    np.testing.assert_array_equal(v, exp["virgin"])
    # idempotence: the same batch again finds nothing new and leaves the virgin map alone
    out2 = ctx.triage(t, oc, WANT_H32)
    torch.cuda.synchronize()
    assert int(out2["hnb"].max()) == 0
    np.testing.assert_array_equal(ctx.get_virgin(), v)


def _run_shards(ctxs, shards, ocs, mode, device, fused=False):
    """One sharded batch over in-process 'ranks' (one context each, same GPU), phase by phase
    as killerbeez_amd.dist.triage_sharded runs them, with the all-gathers done locally.
    fused: the round-6 steps (shard_exchange_row, shard_reduce_into, shard_finish_gathered)."""
    import torch

    world = len(ctxs)
    counts = [s.shape[0] for s in shards]
    outs = [c.shard_begin(s, o, WANT_H32) for c, s, o in zip(ctxs, shards, ocs)]
    nonempty = [r for r in range(world) if counts[r] > 0]
    if mode == MODE_DYNAMORIO:
        m = ctxs[0].map_size
        if fused:
            bufs = torch.stack([c.shard_exchange_row(torch.zeros(m + 16, dtype=torch.uint8,
                                                                 device=device)) for c in ctxs])
            rows, pairs = bufs[:, :m], bufs[:, m:m + 8].contiguous().view(torch.int32)
            # the one-launch exchange equals the two copies it replaces
            for r, c in enumerate(ctxs):
                p2 = c.shard_last_hash(torch.empty(2, dtype=torch.int32, device=device))
                assert torch.equal(p2, pairs[r])
                if counts[r]:
                    r2 = c.shard_last_row(torch.zeros(m, dtype=torch.uint8, device=device))
                    assert torch.equal(r2, rows[r])
        else:
            pairs = torch.stack([c.shard_last_hash(torch.empty(2, dtype=torch.int32,
                                                               device=device)) for c in ctxs])
            rows = torch.stack([c.shard_last_row(torch.zeros(m, dtype=torch.uint8,
                                                             device=device)) for c in ctxs])
        for r, c in enumerate(ctxs):
            prev = [q for q in nonempty if q < r]
            p = prev[-1] if prev else None
            g = nonempty[-1] if nonempty else None
            c.shard_link(None if p is None else pairs[p], None if p is None else rows[p],
                         not prev, None if g is None else pairs[g],
                         None if g is None else rows[g])
    else:
        for c in ctxs:
            c.shard_link(None, None, True, None, None)
    nb = ctxs[0].shard_aggregate_bytes()
    if fused:
        allagg = torch.empty(world, nb, dtype=torch.uint8, device=device)
        for r, c in enumerate(ctxs):
            c.shard_reduce_into(allagg[r])
        res = [c.shard_finish_gathered(allagg, r, world) for r, c in enumerate(ctxs)]
        torch.cuda.synchronize()
        for c in ctxs:
            c.sync()
        return (np.concatenate([o["hnb"].cpu().numpy() for o in res]),
                np.concatenate([o["h32"].cpu().numpy().view(np.uint32) for o in res]))
    for c in ctxs:
        c.shard_reduce()
    allagg = torch.stack([c.shard_aggregate(torch.empty(nb, dtype=torch.uint8, device=device))
                          for c in ctxs])
    res = []
    for r, c in enumerate(ctxs):
        # the fused prefix / total pass (kbz_or_prefix_total) against two kbz_or_reduce launches
        total = torch.empty(nb, dtype=torch.uint8, device=device)
        prefix = torch.empty(nb, dtype=torch.uint8, device=device) if r > 0 else None
        TriageContext.or_prefix_total(prefix, total, allagg, r, world, nb)
        t2 = torch.empty(nb, dtype=torch.uint8, device=device)
        TriageContext.or_reduce(t2, allagg, 0, world, nb)
        assert torch.equal(t2, total)
        if r > 0:
            TriageContext.or_reduce(t2, allagg, 0, r, nb)
            assert torch.equal(t2, prefix)
        res.append(c.shard_finish(prefix, total))
    torch.cuda.synchronize()
    for c in ctxs:
        c.sync()
    return (np.concatenate([o["hnb"].cpu().numpy() for o in res]),
            np.concatenate([o["h32"].cpu().numpy().view(np.uint32) for o in res]))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("counts", [[700, 324], [640, 0, 193, 64]])
@pytest.mark.parametrize("fused", [False, True], ids=["staged-finish", "fused-finish"])
def test_sharded_protocol_on_gpu(gpu, mode, counts, fused):
    """The multi-GPU protocol (dist.py) through the C ABI: shard aggregates (restricted to
    still-virgin bits), prefix/total ORs and the last-hash links give the sequential result,
    batch after batch (the second batch adds new coverage to carried virgin maps)."""
    import torch

    m = 4096
    n = sum(counts)
    ctxs = [TriageContext(m, mode, max(c, 1)) for c in counts]
    v = np.full((3, m), 0xFF, np.uint8)
    last = 0
    for batch in range(3):
        t, oc = synth.sparse_np(n, m, seed=100 + batch, hot_frac=0.05)
        t[300] = t[299]          # DynamoRIO skips inside and across shards
        t[counts[0]] = t[counts[0] - 1]
        exp = oracle.triage_batch(mode, t, oc, virgin=v, last_hash=last, want=oracle.WANT_H32)
        lo, shards, ocs = 0, [], []
        for c in counts:
            shards.append(torch.from_numpy(t[lo:lo + c].copy()).cuda())
            ocs.append(torch.from_numpy(oc[lo:lo + c].copy()).cuda())
            lo += c
        hnb, h32 = _run_shards(ctxs, shards, ocs, mode, torch.device("cuda"), fused)
        np.testing.assert_array_equal(hnb, exp["hnb"])
        np.testing.assert_array_equal(h32, exp["h32"])
        for c in ctxs:
            np.testing.assert_array_equal(c.get_virgin(), exp["virgin"])
            if mode == MODE_DYNAMORIO:
                assert c.last_hash == exp["last_hash"]
        v, last = exp["virgin"], exp.get("last_hash", 0)
        assert batch == 0 or 0 < (hnb > 0).sum() < n  # later batches still find something


@pytest.mark.parametrize("fused", [False, True], ids=["staged-finish", "fused-finish"])
def test_sharded_protocol_collisions(gpu, fused):
    """DynamoRIO shards with ignore bytes: hash collisions (equal hash32_with_ignore, different
    examined bytes) inside a shard, at a shard's row 0 against the previous shard's last row,
    and a chain of repeats of a collided row across a chunk boundary -- the fix path and the
    chain walks of k_chain / k_total ahead of either finish."""
    import torch

    m = 4096
    rng = np.random.default_rng(3121)
    counts = [300, 257, 200]
    n = sum(counts)
    ign = np.where(rng.random(m) < 0.4, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
    zc = np.nonzero(ign == 0)[0]
    ctxs = [TriageContext(m, MODE_DYNAMORIO, c) for c in counts]
    for c in ctxs:
        c.set_ignore(ign)
    v = np.full((3, m), 0xFF, np.uint8)
    last = 0
    for batch in range(2):
        t, oc = synth.sparse_np(n, m, seed=3122 + batch, hot_frac=0.05)
        for j in (50, counts[0], counts[0] + counts[1] + 64):
            _collide(t, j, zc, rng)             # inside, at shard 1's row 0, at a chunk start
        _collide(t, counts[0] + 100, zc, rng)
        t[counts[0] + 101:counts[0] + 140] = t[counts[0] + 100]  # a chain over a chunk boundary
        exp = oracle.triage_batch(MODE_DYNAMORIO, t, oc, virgin=v, ignore=ign, last_hash=last,
                                  want=oracle.WANT_H32)
        lo, shards, ocs = 0, [], []
        for c in counts:
            shards.append(torch.from_numpy(t[lo:lo + c].copy()).cuda())
            ocs.append(torch.from_numpy(oc[lo:lo + c].copy()).cuda())
            lo += c
        hnb, h32 = _run_shards(ctxs, shards, ocs, MODE_DYNAMORIO, torch.device("cuda"), fused)
        np.testing.assert_array_equal(hnb, exp["hnb"])
        np.testing.assert_array_equal(h32, exp["h32"])
        for c in ctxs:
            np.testing.assert_array_equal(c.get_virgin(), exp["virgin"])
            assert c.last_hash == exp["last_hash"]
        v, last = exp["virgin"], exp["last_hash"]


@pytest.mark.parametrize("commit", [False, True], ids=["submit-copies", "early-commits"])
@pytest.mark.parametrize("mode", MODES)
def test_ingest_ring(gpu, mode, commit):
    """kbz_ring_*: the producer writes rows into pinned slots, batches are queued back to back
    (results delivered on re-acquire / flush) and equal one sequential pass over all traces.
    early-commits: rows are written in pieces and kbz_ring_commit starts each piece's copy
    (17-row pieces: a small batch with committed rows goes through device memory; a commit of
    every row, of none, and a repeated commit)."""
    m, sizes = 4096, [300, 17, 0, 256, 1, 300]
    ctx = TriageContext(m, mode, 300)
    t, oc = synth.sparse_np(sum(sizes), m, seed=77, hot_frac=0.05)
    t[301] = t[300]  # DynamoRIO skip across a batch boundary
    oc[300:317] = oracle.FUZZ_NONE  # batch 1 is submitted without an outcome array
    exp = oracle.triage_batch(mode, t, oc, virgin=ctx.get_virgin(), last_hash=ctx.last_hash,
                              want=oracle.WANT_H32 | oracle.WANT_X64)
    outs, lo = [], 0
    for i, n in enumerate(sizes):
        rows, ocs = ctx.ring_acquire()
        assert rows.shape[0] >= n and rows.shape[1] == m
        if commit:
            ctx.ring_commit(0)
            for a in range(0, n, 17):
                b = min(n, a + 17)
                rows[a:b] = t[lo + a:lo + b]
                if b < n or i % 2:  # odd batches commit every row, even ones leave a tail
                    ctx.ring_commit(b)
                    ctx.ring_commit(b)
        else:
            rows[:n] = t[lo:lo + n]
        ocs[:n] = oc[lo:lo + n]
        hnb = np.full(n, 0xEE, np.uint8)
        h32 = np.zeros(n, np.uint32)
        x64 = np.zeros(n, np.uint64)
        if i == 1:
            ocs[:n] = -7  # stale slot contents must not be read without have_outcome
        ctx.ring_submit(n, i != 1, hnb, h32, x64, WANT_H32 | WANT_X64)
        outs.append((lo, n, hnb, h32, x64))
        lo += n
    ctx.ring_flush()
    for lo, n, hnb, h32, x64 in outs:
        np.testing.assert_array_equal(hnb, exp["hnb"][lo:lo + n])
        np.testing.assert_array_equal(h32, exp["h32"][lo:lo + n])
        np.testing.assert_array_equal(x64, exp["x64"][lo:lo + n])
    np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])
    if mode == MODE_DYNAMORIO:
        assert ctx.last_hash == exp["last_hash"]
    ctx.close()


@pytest.mark.parametrize("files,iters,size", [(3, 7, 65536), (1, 2, 1 << 20), (2, 1, 4096),
                                              (0, 4, 4096), (70000, 2, 16)])
def test_picker_ignore(gpu, files, iters, size):
    """kbz_picker_ignore_device vs the restated picker diff (picker/main.c:240-262)."""
    import torch

    from killerbeez_amd.triage import picker_ignore

    rng = np.random.default_rng(files + 31 * iters)
    base = rng.integers(0, 256, size=(files, 1, size), dtype=np.uint8)
    runs = np.repeat(base, iters, axis=1)
    noise = rng.random((files, iters, size)) < 0.005
    runs[noise] = rng.integers(0, 256, size=int(noise.sum()), dtype=np.uint8)
    ign, pc, tot = oracle.picker_ignore(runs)
    g_ign, g_pc, g_tot = picker_ignore(torch.from_numpy(runs).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(g_ign.cpu().numpy(), ign)
    np.testing.assert_array_equal(g_pc.cpu().numpy().view(np.uint32), pc)
    assert int(g_tot.item()) == tot


def test_picker_rejects_unaligned_size(gpu):
    import torch

    from killerbeez_amd.triage import picker_ignore

    with pytest.raises(Exception):
        picker_ignore(torch.zeros((1, 2, 24), dtype=torch.uint8, device="cuda"))


def test_triage_modules_per_module_coverage(gpu):
    """kbz_triage_modules_device = has_new_coverage_per_module (dynamorio_instrumentation.c:
    1477-1493): every module keeps its own virgin map / ignore bytes / last hash; the per-exec
    result is the OR over modules.  Two carried batches, 3 modules of different map sizes packed
    in one row, ignore bytes on one module, repeated execs (last-hash skips)."""
    import torch

    from killerbeez_amd.triage import triage_modules

    sizes = [65536, 4096, 16384]
    offs = [0, 65536, 65536 + 4096]
    row = sum(sizes)
    rng = np.random.default_rng(1477)
    ign = np.where(rng.random(4096) < 0.1, 0, 0xFF).astype(np.uint8)
    ctxs = [TriageContext(m, MODE_DYNAMORIO, 300) for m in sizes]
    ctxs[1].set_ignore(ign)
    virgins = [np.full((3, m), 0xFF, np.uint8) for m in sizes]
    lasts = [0] * 3
    for b in range(2):
        n = 300 - 100 * b
        parts = [synth.sparse_np(n, m, seed=10 * b + i)[0] for i, m in enumerate(sizes)]
        for p in parts:
            p[50:60] = p[49]  # identical consecutive execs
        traces = np.concatenate(parts, axis=1)
        hnb, anyv = triage_modules(ctxs, torch.from_numpy(traces).cuda(), offs)
        torch.cuda.synchronize()
        exp_any = np.zeros(n, np.uint8)
        for i, m in enumerate(sizes):
            exp = oracle.triage_batch(MODE_DYNAMORIO, parts[i], None, virgin=virgins[i],
                                      ignore=ign if i == 1 else None, last_hash=lasts[i])
            np.testing.assert_array_equal(hnb[i].cpu().numpy(), exp["hnb"])
            np.testing.assert_array_equal(ctxs[i].get_virgin(), exp["virgin"])
            assert ctxs[i].last_hash == exp["last_hash"]
            virgins[i], lasts[i] = exp["virgin"], exp["last_hash"]
            exp_any |= (exp["hnb"] != 0).astype(np.uint8)
        np.testing.assert_array_equal(anyv.cpu().numpy(), exp_any)
    for c in ctxs:
        c.close()


# ---- at scale: >= 512 chunks, so AUTO picks k_pass1s (the config-2 kernel) ------------------
N_AT_SCALE = 32768 + 37  # 513 chunks, the last one partial


@pytest.mark.parametrize("mode", [MODE_AFL, MODE_AFL_CLASSIFY])
@pytest.mark.parametrize("m", [256, 4096])
@pytest.mark.parametrize("want", [0, WANT_H32, WANT_H32 | WANT_X64], ids=["nohash", "h32", "h32x64"])
def test_at_scale_afl_outcome_routing(gpu, mode, m, want):
    """3 virgin maps (finish_fuzz_round afl_instrumentation.c:231-274): 5 % hangs + crashes go
    simplified to virgin_tmout / virgin_crash, with all-zero traces (simplify's 0x01 words) and
    identical neighbours; XXH64 on; a second batch carries the three maps."""
    t, oc = synth.sparse_np(N_AT_SCALE, m, seed=231 + m + mode, hot_frac=0.05,
                            outcome_p=(0.95, 0.02, 0.03))
    t[100:110] = 0
    t[640:700] = t[639]
    oc[640:700] = oracle.FUZZ_CRASH
    ctx = TriageContext(m, mode, N_AT_SCALE)
    e1 = check(mode, t, oc, ctx=ctx, want=want)
    for k in range(3):
        assert (e1["hnb"][oc == k] > 0).any()
    t2, oc2 = synth.sparse_np(N_AT_SCALE, m, seed=232 + m + mode, hot_frac=0.05,
                              outcome_p=(0.9, 0.05, 0.05))
    check(mode, t2, oc2, ctx=ctx, want=want)
    ctx.close()


def _collide(t, j, zc, rng, k=12):
    """Row j = row j-1 except on k bytes that the ignore map hides from hash32_with_ignore but
    has_new_bits_with_ignore examines: equal hashes, different content (a collision)."""
    t[j] = t[j - 1]
    t[j, rng.choice(zc, k)] = rng.integers(1, 256, k)


def _expected_fix(t, h32, ign, last_hash, prev_row, prev_clean=True):
    """What the skip fix path must recompute (kbz_triage.hip k_skip / k_chain), from first
    principles: skip[j] = h[j] == h[j-1]; a skipped row that differs from its predecessor on
    the examined bytes -- or, for row 0, whose predecessor (the previous batch's last row) is
    unknown or not clean -- is bad; every chunk holding a bad row or a repeat chained to one is
    recomputed.  The batch's last row is then clean (never excluded from V while its repeats
    were applied) by the engine's conservative rule: no bad row j >= 1, and some row j >= 1
    applied or row 0 not bad.  Returns (bad rows j >= 1, recomputed chunks, last row clean)."""
    lut = oracle.count_class_table()
    x = lut[t]
    rel = np.ones(t.shape[1], bool) if ign is None else ign == 0
    n = t.shape[0]
    prevh = np.concatenate([[last_hash], h32[:-1]]).astype(np.uint32)
    skip = h32 == prevh
    differs = np.zeros(n, bool)
    differs[1:] = ((x[1:] != x[:-1]) & rel).any(axis=1)
    differs[0] = (prev_row is None or not prev_clean or
                  ((x[0] != lut[prev_row]) & rel).any())
    bad = skip & differs
    chunks = set()
    for r in np.nonzero(bad)[0]:
        chunks.add(r // 64)
        j = r + 1
        while j < n and skip[j] and not differs[j]:
            if j % 64 == 0:
                chunks.add(j // 64)
            j += 1
    clean = not bad[1:].any() and ((~skip[1:]).any() or not bad[0])
    return int(bad[1:].sum()), chunks, clean


def test_at_scale_dynamorio_repeats_and_collisions(gpu, pass1):
    """has_new_coverage (dynamorio_instrumentation.c:1428-1468) at 513 chunks with ignore bytes:
    exact repeats everywhere, at chunk starts (lane 0, compared with the previous chunk's last
    row), runs over several chunks; collisions inside chunks and at lane 0, one followed by a
    700-row chain of repeats (every chunk the chain enters must be recomputed).  Then batches
    whose row 0 repeats the previous batch's last exec: when that exec was a collision (never
    applied: its repeats must not be applied either), when it was clean (nothing to recompute),
    and when row 0 collides with it (row 0 and its chain are recomputed)."""
    m = 4096
    rng = np.random.default_rng(1428)
    t, oc = synth.sparse_np(N_AT_SCALE, m, seed=1429, hot_frac=0.05)
    ign = np.where(rng.random(m) < 0.4, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
    zc = np.nonzero(ign == 0)[0]
    for c in range(1, 513, 3):
        t[64 * c] = t[64 * c - 1]           # exact repeat at lane 0
    for j in rng.integers(1, N_AT_SCALE, 400):
        t[j] = t[j - 1]                     # exact repeats anywhere
    t[5000:5300] = t[4999]                  # a run over several chunks
    for j in [64 * 7, 64 * 11, 777, 5555, 20001, N_AT_SCALE - 1]:
        _collide(t, j, zc, rng)
    _collide(t, 9000, zc, rng)              # a collision, then a chain of repeats of it
    t[9001:9700] = t[9000]
    ctx = TriageContext(m, MODE_DYNAMORIO, N_AT_SCALE)
    ctx.set_ignore(ign)
    exp = check(MODE_DYNAMORIO, t, oc, ignore=ign, ctx=ctx)
    nbad, chunks, clean = _expected_fix(t, exp["h32"], ign, 0, None)
    assert nbad >= 7 and set(range(141, 152)) <= chunks and len(chunks) < 40 and not clean
    st = ctx.stats()
    assert (st["fixed_chunks"], st["bad_rows"]) == (len(chunks), nbad)
    last, prev = exp["last_hash"], t[-1].copy()
    batches = []
    t2, oc2 = synth.sparse_np(4000, m, seed=1430, hot_frac=0.05)
    t2[0] = t[-1]                           # repeats the last exec, a collision (not clean)
    t2[1:300] = t2[0]
    batches.append((t2, {0, 1, 2, 3, 4}))
    t3 = t2.copy()
    t3[0] = t2[-1]
    t3[0, rng.choice(zc, 12)] = rng.integers(1, 256, 12)  # collides with the (clean) last exec
    t3[1:200] = t3[0]
    batches.append((t3, {0, 1, 2, 3}))
    t4 = synth.sparse_np(4000, m, seed=1431, hot_frac=0.05)[0]
    t4[0] = t3[-1]                          # repeats the (clean) last exec: nothing to redo
    t4[1:100] = t4[0]
    batches.append((t4, set()))
    for tb, want_chunks in batches:
        e = check(MODE_DYNAMORIO, tb, oc2, ignore=ign, ctx=ctx)
        assert e["hnb"][0] == 0
        nb, ch, cl = _expected_fix(tb, e["h32"], ign, last, prev, clean)
        assert ch == want_chunks and nb == 0
        st = ctx.stats()
        assert (st["fixed_chunks"], st["bad_rows"]) == (len(ch), nb)
        last, prev, clean = e["last_hash"], tb[-1].copy(), cl
    ctx.close()


def test_dynamorio_restored_hash_unknown_predecessor(gpu):
    """kbz_set_last_hash (state restore) forgets the previous trace: a repeated first exec is
    then handled without it -- row 0 and its chain of repeats (3 chunks) are recomputed."""
    m = 4096
    t, oc = synth.sparse_np(40000, m, seed=1461, hot_frac=0.05)
    t[1:150] = t[0]
    exp_h0 = oracle.triage_batch(MODE_DYNAMORIO, t[:1], None)["h32"][0]
    ctx = TriageContext(m, MODE_DYNAMORIO, 40000)
    ctx.last_hash = int(exp_h0)
    exp = check(MODE_DYNAMORIO, t, oc, ctx=ctx)
    assert exp["hnb"][0] == 0
    assert ctx.stats()["fixed_chunks"] == 3
    ctx.close()


@pytest.mark.parametrize("with_ignore", [False, True])
def test_lookback_timeout_recomputes_predecessor_hash(gpu, monkeypatch, with_ignore):
    """k_pass1s's fused skip rule with a look-back that gives up at once
    (KBZ_DEBUG_LOOKBACK_SPIN=0): a chunk whose lower neighbour has not published yet recomputes
    that neighbour's last-row hash from the row (hash32 / hash32_with_ignore of the classified
    map) instead of using a stale word.  Results stay exact; the stall is reported as flag 0x200
    when it happened."""
    import torch

    from killerbeez_amd._lib import KbzError

    monkeypatch.setenv("KBZ_DEBUG_LOOKBACK_SPIN", "0")
    m = 4096
    rng = np.random.default_rng(4411)
    t, oc = synth.sparse_np(N_AT_SCALE, m, seed=4412, hot_frac=0.05)
    ign = None
    if with_ignore:
        ign = np.where(rng.random(m) < 0.4, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
        _collide(t, 64 * 9, np.nonzero(ign == 0)[0], rng)  # a collision at a chunk start
    for c in range(1, 513, 2):
        t[64 * c] = t[64 * c - 1]           # repeats at chunk starts: row 0's rule decides
    exp = oracle.triage_batch(MODE_DYNAMORIO, t, oc, ignore=ign, want=oracle.WANT_H32)
    with TriageContext(m, MODE_DYNAMORIO, N_AT_SCALE) as ctx:
        if ign is not None:
            ctx.set_ignore(ign)
        out = ctx.triage(torch.from_numpy(t).cuda(), torch.from_numpy(oc).cuda(), WANT_H32)
        torch.cuda.synchronize()
        try:
            ctx.sync()
        except KbzError as e:
            assert "0x200" in str(e), e
        np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
        np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), exp["h32"])
        np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])
        assert ctx.last_hash == exp["last_hash"]


@pytest.mark.parametrize("mode", MODES)
def test_at_scale_x64_partial_chunk(gpu, mode):
    m = 256
    t, oc = synth.sparse_np(N_AT_SCALE, m, seed=855 + mode, hot_frac=0.1)
    check(mode, t, oc, want=WANT_H32 | WANT_X64)


@pytest.mark.parametrize("mode", MODES)
def test_abandoned_batch_is_rearmed(gpu, mode):
    """A batch abandoned between the sharded stages (e.g. a failed collective) leaves per-batch
    state behind; the next kbz_shard_begin re-arms it and the next batch is exact."""
    import torch

    m = 4096
    t, oc = synth.sparse_np(3000, m, seed=1593, hot_frac=0.05)
    t[64] = t[63]
    ctx = TriageContext(m, mode, 3000)
    v0, l0 = ctx.get_virgin(), ctx.last_hash
    tt, oo = torch.from_numpy(t).cuda(), torch.from_numpy(oc).cuda()
    ctx.shard_begin(tt, oo, WANT_H32)
    ctx.shard_link(None, None, True, None, None)
    ctx.shard_reduce()
    torch.cuda.synchronize()                # abandoned here: no shard_finish
    ctx.set_virgin(v0)
    ctx.last_hash = l0
    small = t[:500]
    check(mode, small, oc[:500], ctx=ctx)
    ctx.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("want", [0, WANT_H32 | WANT_X64], ids=["nohash", "hashes"])
def test_config3_dense_1m(gpu, mode, want):
    """BASELINE config 3's traces (dense: 50 % hot, counts U[1,255]) at 1 MiB, at a batch size
    the sequential oracle checks in seconds, crash/hang mixed in."""
    t, oc = synth.dense_np(300, 1 << 20, seed=3 + mode, outcome_p=(0.8, 0.1, 0.1))
    t[65] = t[64]
    check(mode, t, oc, want=want)


@pytest.mark.slow
def test_full_size_config3(gpu):
    """BASELINE config 3 at full size: 16,384 dense traces x 1 MiB (16 GiB), DynamoRIO mode,
    exactly against the sharded CPU oracle, then idempotence."""
    import torch

    n, m = 16384, 1 << 20
    t, oc = synth.dense_torch(n, m, seed=0x5EED, device="cuda")
    ctx = TriageContext(m, MODE_DYNAMORIO, n)
    out = ctx.triage(t, oc, WANT_H32)
    torch.cuda.synchronize()
    ctx.sync()
    th = t.cpu().numpy()
    exp = oracle.triage_batch(MODE_DYNAMORIO, th, oc.cpu().numpy(), threads=16)
    del th
    np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
    np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), exp["h32"])
    v = ctx.get_virgin()
    np.testing.assert_array_equal(v, exp["virgin"])
    out2 = ctx.triage(t, oc, WANT_H32)
    torch.cuda.synchronize()
    assert int(out2["hnb"].max()) == 0
    np.testing.assert_array_equal(ctx.get_virgin(), v)
    ctx.close()


@pytest.mark.parametrize("xf", [0, 1, 2])
def test_transform_rows(gpu, xf):
    """kbz_transform_rows_device: classify_counts / simplify_trace of every row (the maps
    get_module_info and dump_map_dir hand out), strided rows, against the restatement."""
    import torch

    from killerbeez_amd.triage import transform_rows

    t = synth.uniform_np(300, 4096, seed=xf, density=0.3)
    t[5] = 0
    big = torch.zeros((300, 4096 + 256), dtype=torch.uint8, device="cuda")
    big[:, :4096] = torch.from_numpy(t).cuda()
    got = transform_rows(big[:, :4096], xf)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), oracle.transform(t, xf))


def test_set_virgin_after_a_batch_forgets_the_saved_row(gpu):
    """A batch ends in row R; the virgin maps are then replaced (kbz_set_virgin) with the last
    hash kept; the next batch starts with R again (a last-hash skip: never applied) and then a
    row holding R's edges, which is new against the fresh maps.  The saved row may no longer
    be taken as already absorbed."""
    m = 4096
    t, oc = synth.sparse_np(200, m, seed=2045, hot_frac=0.05)
    ctx = TriageContext(m, MODE_DYNAMORIO, 200)
    check(MODE_DYNAMORIO, t[:100], oc[:100], ctx=ctx)
    fresh = np.full((3, m), 0xFF, np.uint8)
    ctx.set_virgin(fresh)
    t2 = t[100:].copy()
    t2[0] = t[99]
    t2[1] = t[99]
    t2[1, 7] ^= 0x01                                  # R's edges plus a changed byte
    exp = check(MODE_DYNAMORIO, t2, oc[100:], ctx=ctx)
    assert exp["hnb"][0] == 0 and exp["hnb"][1] == 2
    ctx.close()


@pytest.mark.parametrize("mode", MODES)
def test_reset_virgin_is_stream_ordered(gpu, mode):
    """kbz_reset_virgin between two batches enqueued back to back (no host sync): the second
    batch sees all-0xff maps, the DynamoRIO last hash carries over, and its first rows repeat
    the first batch's last row (a skip, then a changed copy that is new again)."""
    import torch

    m = 4096
    t, oc = synth.sparse_np(300, m, seed=2031 + mode, hot_frac=0.05)
    a, b = t[:150].copy(), t[150:].copy()
    b[0] = a[-1]
    b[1] = a[-1]
    b[1, 11] ^= 0x02
    fresh = np.full((3, m), 0xFF, np.uint8)
    exp_a = oracle.triage_batch(mode, a, oc[:150], virgin=fresh, want=oracle.WANT_H32)
    exp_b = oracle.triage_batch(mode, b, oc[150:], virgin=fresh, last_hash=exp_a["last_hash"],
                                want=oracle.WANT_H32)
    with TriageContext(m, mode, 150) as ctx:
        ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
        oa, ob = torch.from_numpy(oc[:150]).cuda(), torch.from_numpy(oc[150:]).cuda()
        ra = ctx.triage(ta, oa, WANT_H32)
        ctx.reset_virgin()
        rb = ctx.triage(tb, ob, WANT_H32)
        torch.cuda.synchronize()
        ctx.sync()
        np.testing.assert_array_equal(ra["hnb"].cpu().numpy(), exp_a["hnb"])
        np.testing.assert_array_equal(rb["hnb"].cpu().numpy(), exp_b["hnb"])
        np.testing.assert_array_equal(rb["h32"].cpu().numpy().view(np.uint32), exp_b["h32"])
        np.testing.assert_array_equal(ctx.get_virgin(), exp_b["virgin"])
        if mode == MODE_DYNAMORIO:
            assert ctx.last_hash == exp_b["last_hash"]
            assert exp_b["hnb"][0] == 0 and exp_b["hnb"][1] > 0


@pytest.mark.parametrize("path", ["host", "ring"])
@pytest.mark.parametrize("mode", MODES)
def test_reset_virgin_then_host_batch(gpu, mode, path):
    """kbz_reset_virgin on the caller's stream (torch's current stream, held busy by a long
    kernel so the fill lands late), then a host batch (kbz_triage_batch_host) or a ring submit:
    both run on the context's own non-blocking stream, which must wait for the fill.  And the
    other order: a ring batch still queued when the reset is issued is not overwritten by it."""
    import torch

    m = 4096
    t, oc = synth.sparse_np(300, m, seed=2087 + mode, hot_frac=0.05)
    a, b = t[:150].copy(), t[150:].copy()
    fresh = np.full((3, m), 0xFF, np.uint8)
    exp_a = oracle.triage_batch(mode, a, oc[:150], virgin=fresh, want=oracle.WANT_H32)
    exp_b = oracle.triage_batch(mode, b, oc[150:], virgin=fresh, last_hash=exp_a["last_hash"],
                                want=oracle.WANT_H32)
    with TriageContext(m, mode, 150) as ctx:
        if path == "host":
            ra = ctx.triage_host(a, oc[:150], WANT_H32)
        else:
            rows, roc = ctx.ring_acquire()
            rows[:150] = a
            roc[:150] = oc[:150]
            ra = {"hnb": np.zeros(150, np.uint8)}
            ctx.ring_submit(150, True, ra["hnb"])  # still queued when the reset is issued
        torch.cuda._sleep(50_000_000)  # ~20 ms of GPU time ahead of the fill on this stream
        ctx.reset_virgin()
        if path == "host":
            rb = ctx.triage_host(b, oc[150:], WANT_H32)
        else:
            rows, roc = ctx.ring_acquire()
            rows[:150] = b
            roc[:150] = oc[150:]
            rb = {"hnb": np.zeros(150, np.uint8)}
            ctx.ring_submit(150, True, rb["hnb"])
            ctx.ring_flush()
        torch.cuda.synchronize()
        ctx.sync()
        np.testing.assert_array_equal(ra["hnb"], exp_a["hnb"])
        np.testing.assert_array_equal(rb["hnb"], exp_b["hnb"])
        np.testing.assert_array_equal(ctx.get_virgin(), exp_b["virgin"])
        if mode == MODE_DYNAMORIO:
            assert ctx.last_hash == exp_b["last_hash"]


def test_claim_overflow_is_reported_once(gpu, monkeypatch):
    """A claim-list overflow (forced with a tiny debug list) fails that batch once: the next
    ring acquire / record works and later batches are exact again."""
    from killerbeez_amd import plugin as P

    monkeypatch.setenv("KBZ_DEBUG_ITEM_CAP", "16")
    monkeypatch.setenv("KBZ_DEBUG_WIN_ITEMS", "1")  # every claimed window an item (k_scan would
    m = 4096                                         # resolve windows of few claims itself)
    t, oc = synth.sparse_np(300, m, seed=2529, hot_frac=0.05)
    p = P.Plugin("afl_gpu", '{"map_size": %d, "max_batch": 256}' % m)
    with pytest.raises(RuntimeError, match="overflow"):
        p.triage_batch(t[:200], oc[:200])            # fresh maps: far more than 16 claims
    v = P.state_maps(p.get_state(), m)
    vm = np.stack([v["virgin_bits"], v["virgin_tmout"], v["virgin_crash"]])
    one = np.zeros((1, m), np.uint8)
    one[0, 11] = 3                                   # a new edge: a handful of claims
    for j, row in enumerate([t[200], one[0], t[201]]):
        tk = p.record(row, P.FUZZ_NONE)
        assert tk >= 0, P.last_error()
        rows = np.stack([t[200], one[0], t[201]])[:j + 1]
        exp = oracle.triage_batch(MODE_AFL, rows, np.zeros(j + 1, np.int8), virgin=vm)
        assert p.result(tk) == exp["hnb"][j]


@pytest.mark.parametrize("inl", [None, "0", "1000000"], ids=["inline16", "inline0", "inline-all"])
@pytest.mark.parametrize("win", ["1", "16", "1000000"], ids=["all-windows", "default", "no-windows"])
@pytest.mark.parametrize("mode", MODES)
def test_claims_window_and_byte_items(gpu, mode, win, inl, monkeypatch):
    """The claim paths give identical results: k_scan resolving a window's few claimed bytes
    itself (one byte of each of the chunk's rows per claim, 8 claims per round trip; the
    per-byte items of KBZ_SCAN_INLINE=0 builds follow the same rule in k_resolve) and window
    items (k_resolve streams the chunk's 1-KiB column window row by row in order).  Fresh virgin maps and dense rows make windows with hundreds of
    claimed bytes, sparse rows windows with one or two; a 4,864-B map leaves lanes of its last window
    past the end; partial last chunk; DynamoRIO with ignore bytes and repeated execs (skipped
    rows must not claim), AFL with hangs/crashes (simplified classes: every byte claims)."""
    monkeypatch.setenv("KBZ_DEBUG_WIN_ITEMS", win)
    if inl is not None:  # the fused tail's inline-claim budget per wave (the rest: byte items)
        monkeypatch.setenv("KBZ_DEBUG_TAIL_INLINE_MAX", inl)
    rng = np.random.default_rng(int(win) % 97 + mode)
    for m, n in [(65536, 700), (19 * 256, 200), (1 << 20, 70)]:
        t = synth.uniform_np(n, m, seed=m + n, density=0.3)
        t[: n // 3] = synth.uniform_np(n // 3, m, seed=m - n, density=0.01)
        oc = rng.choice(3, size=n, p=[0.8, 0.1, 0.1]).astype(np.int8)
        ign = None
        if mode == MODE_DYNAMORIO:
            ign = np.where(rng.random(m) < 0.7, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
            for j in rng.integers(1, n, n // 4):
                t[j] = t[j - 1]                # skipped rows (same hash): never claim
        ctx = TriageContext(m, mode, n)
        if ign is not None:
            ctx.set_ignore(ign)
        exp = check(mode, t, oc, ignore=ign, ctx=ctx)
        assert exp["hnb"].max() == 2
        t2 = synth.uniform_np(n, m, seed=m + 2 * n, density=0.3)
        check(mode, t2, oc, ignore=ign, ctx=ctx)  # carried maps: fewer, scattered claims
        ctx.close()
