"""The fused one-shard tail (k_skip with its row-0 / saved-row roles + k_tail) at grid sizes far
beyond what the GPU holds at once: a 1 MiB map makes k_tail's grid 256 column groups x up to 32
segments, so its waits (the chain walks' flag, each column group's fix flag) are on workgroups of
lower linear index that must have been dispatched first.  DynamoRIO with ignore bytes and hash
collisions (the fix path), window items (fresh maps), and the same batches through the staged
kernels for comparison; every result against the oracle."""
import numpy as np
import pytest

import oracle
from killerbeez_amd import synth
from killerbeez_amd.triage import MODE_AFL, MODE_DYNAMORIO, WANT_H32, TriageContext

from tests.test_gpu_parity import _collide, check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("staged", [False, True], ids=["fused", "staged"])
def test_tail_1mib_collisions(gpu, staged, monkeypatch):
    if staged:
        monkeypatch.setenv("KBZ_DEBUG_STAGED", "1")
    m, n = 1 << 20, 64 * 33 + 5
    rng = np.random.default_rng(1300)
    t, oc = synth.sparse_np(n, m, seed=1301, hot_frac=0.02)
    ign = np.where(rng.random(m) < 0.4, 0, rng.integers(1, 256, size=m)).astype(np.uint8)
    zc = np.nonzero(ign == 0)[0]
    for j in (64, 700, 1500):
        _collide(t, j, zc, rng)
    t[701:900] = t[700]  # a chain of repeats after a collision: several chunks recomputed
    with TriageContext(m, MODE_DYNAMORIO, n) as ctx:
        ctx.set_ignore(ign)
        e = check(MODE_DYNAMORIO, t, oc, ignore=ign, ctx=ctx)  # fresh maps: window items
        assert (e["hnb"] == 2).any()
        assert ctx.stats()["bad_rows"] >= 3 and ctx.stats()["fixed_chunks"] >= 4
        t2, oc2 = synth.sparse_np(n, m, seed=1302, hot_frac=0.02)
        t2[0] = t[-1]
        t2[1:80] = t2[0]
        check(MODE_DYNAMORIO, t2, oc2, ignore=ign, ctx=ctx)


@pytest.mark.parametrize("staged", [False, True], ids=["fused", "staged"])
def test_tail_afl_three_maps_large_grid(gpu, staged, monkeypatch):
    if staged:
        monkeypatch.setenv("KBZ_DEBUG_STAGED", "1")
    m, n = 1 << 20, 64 * 20 + 3
    t, oc = synth.sparse_np(n, m, seed=1310, hot_frac=0.02, outcome_p=(0.8, 0.1, 0.1))
    with TriageContext(m, MODE_AFL, n) as ctx:
        check(MODE_AFL, t, oc, ctx=ctx, want=WANT_H32)
        t2, oc2 = synth.sparse_np(n, m, seed=1311, hot_frac=0.02, outcome_p=(0.8, 0.1, 0.1))
        check(MODE_AFL, t2, oc2, ctx=ctx, want=0)


def test_tail_touched_rows_only(gpu):
    """hnb_out rows the tail never scores are written 0 (k_fin copies every row of hnb32, which
    the previous batch's k_fin re-armed): a batch in which only a few rows bring anything new,
    after a warm-up batch, with garbage in the output buffer."""
    import torch

    m = 65536
    t, oc = synth.sparse_np(5000, m, seed=1320, hot_frac=0.05)
    with TriageContext(m, MODE_DYNAMORIO, 5000) as ctx:
        check(MODE_DYNAMORIO, t, oc, ctx=ctx)
        t2 = t.copy()
        t2[[17, 1234, 4321]] = np.random.default_rng(1).integers(0, 256, (3, m), dtype=np.uint8)
        exp = oracle.triage_batch(MODE_DYNAMORIO, t2, oc, virgin=ctx.get_virgin(),
                                  last_hash=ctx.last_hash)
        out = {"hnb": torch.full((5000,), 7, dtype=torch.uint8, device="cuda")}
        ctx.triage(torch.from_numpy(t2).cuda(), torch.from_numpy(oc).cuda(), WANT_H32, out=out)
        torch.cuda.synchronize()
        ctx.sync()
        np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
        assert set(np.nonzero(exp["hnb"])[0]) <= {17, 1234, 4321}


@pytest.mark.parametrize("rec", [True, False], ids=["records", "rows"])
def test_claim_records_fresh_batches(gpu, rec, monkeypatch):
    """Pass-1 claim records (k_pass1s, DynamoRIO, hash32 only): a warm map, then fresh batches of
    the same target (slices of one generated run: one hot set) with repeated execs and a restored
    last hash (row 0 skipped with an unknown predecessor: its chunk goes to the fix list) -- the
    records path for tiles with few still-virgin words, the row reads for the rest and for
    fix-list chunks; against the oracle, and the same batches with records off."""
    if not rec:
        monkeypatch.setenv("KBZ_DEBUG_NO_REC", "1")
    m, n, nb = 16384, 64 * 40 + 17, 6
    t_all, oc_all = synth.sparse_np(n * nb, m, seed=1401, hot_frac=0.02)
    with TriageContext(m, MODE_DYNAMORIO, n, pass1="narrow") as ctx:
        for i in range(nb):
            t, oc = t_all[i * n:(i + 1) * n].copy(), oc_all[i * n:(i + 1) * n]
            if i >= 2:
                t[100:140] = t[99]  # repeats: link rows (skipped, same bytes)
                t[700:705] = t[700]
            if i == 4:  # a restored hash equal to row 0's: row 0 and its repeats are recomputed
                t[1:70] = t[0]
                ctx.last_hash = int(oracle.triage_batch(MODE_DYNAMORIO, t[:1], None)["h32"][0])
            e = check(MODE_DYNAMORIO, t, oc, ctx=ctx, want=WANT_H32)
            if i == 4:
                assert ctx.stats()["fixed_chunks"] >= 2
            if i >= 1:
                assert 0 < (e["hnb"] > 0).sum() < n // 2  # a warm map: some rows are new
