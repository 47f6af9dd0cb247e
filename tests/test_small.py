"""k_small: AFL-mode batches of at most 64 execs without hashes in one launch (the AFL plugin's
per-exec flushes, fuzzer/main.c:385).  Bit-exact with the oracle over sequences of small batches
(outcome routing to the three virgin maps, afl_instrumentation.c:231-274; has_new_bits
:600-662), map sizes 256 B - 1 MiB, interleaved with batches through the general pipeline on the
same context, and with the general pipeline forced for the same batches."""
import numpy as np
import pytest

import oracle
from killerbeez_amd import synth
from killerbeez_amd.triage import MODE_AFL, MODE_AFL_CLASSIFY, WANT_H32, TriageContext

from tests.test_gpu_parity import gpu_triage

pytestmark = pytest.mark.gpu
AFL_MODES = [MODE_AFL, MODE_AFL_CLASSIFY]


def _rows(n, m, seed):
    t, oc = synth.sparse_np(n, m, seed=seed, hot_frac=0.05, outcome_p=(0.7, 0.15, 0.15))
    rng = np.random.default_rng(seed)
    t[3] = 0                                     # an all-zero row (simplified: all 0x01)
    t[7] = t[6]                                  # a repeated exec
    t[11] = rng.integers(0, 256, m, dtype=np.uint8)  # a dense row
    return t, oc


def _run(ctx, mode, t, oc, want=0):
    v0 = ctx.get_virgin()
    exp = oracle.triage_batch(mode, t, oc, virgin=v0, want=oracle.WANT_H32)
    got = gpu_triage(ctx, t, oc, want)
    np.testing.assert_array_equal(got["hnb"], exp["hnb"])
    np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])
    return exp


@pytest.mark.parametrize("mode", AFL_MODES)
@pytest.mark.parametrize("m", [256, 4096, 65536, 1 << 20])
def test_small_batch_sequence(gpu, mode, m):
    sizes = [1, 2, 64, 63, 17, 1, 1, 33, 16, 5]
    t, oc = _rows(sum(sizes), m, seed=m + mode)
    rng = np.random.default_rng(m)
    with TriageContext(m, mode, 64) as ctx:
        v = np.full((3, m), 0xFF, np.uint8)
        msk = rng.random((3, m)) < 0.3
        v[msk] = rng.integers(0, 256, int(msk.sum()), dtype=np.uint8)
        ctx.set_virgin(v)
        lo, twos = 0, 0
        for s in sizes:
            exp = _run(ctx, mode, t[lo:lo + s], oc[lo:lo + s])
            twos += int((exp["hnb"] == 2).sum())
            lo += s
            assert ctx.stats()["claims"] == 0
        assert twos > 0


@pytest.mark.parametrize("mode", AFL_MODES)
def test_small_interleaved_with_general(gpu, mode):
    """Small batches, a 300-exec batch and a hashed small batch (both through the general
    pipeline), small again: one carried virgin state."""
    m = 65536
    t, oc = _rows(64 + 300 + 40 + 9 + 1, m, seed=5 + mode)
    with TriageContext(m, mode, 300) as ctx:
        _run(ctx, mode, t[:64], oc[:64])
        _run(ctx, mode, t[64:364], oc[64:364])
        _run(ctx, mode, t[364:404], oc[364:404], want=WANT_H32)
        _run(ctx, mode, t[404:413], oc[404:413])
        _run(ctx, mode, t[413:], None)  # no outcome array: every exec a FUZZ_NONE


@pytest.mark.parametrize("mode", AFL_MODES)
def test_small_matches_general_pipeline(gpu, mode, monkeypatch):
    m = 16384
    t, oc = _rows(64, m, seed=9 + mode)
    with TriageContext(m, mode, 64) as ctx:
        a = gpu_triage(ctx, t, oc, 0)["hnb"]
        va = ctx.get_virgin()
    monkeypatch.setenv("KBZ_DEBUG_NO_SMALL", "1")
    with TriageContext(m, mode, 64) as ctx:
        b = gpu_triage(ctx, t, oc, 0)["hnb"]
        vb = ctx.get_virgin()
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(va, vb)
