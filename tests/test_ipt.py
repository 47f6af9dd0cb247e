"""Intel-PT path keys and novelty (linux_ipt_instrumentation.c:115-189,
:238-243, :409-424, state :986-1080, merge :944-978).

CPU: the clean-room restatement (oracle kbzo_ipt_keys) reproduces tests/golden/ipt.npz, whose
keys come from the reference's own feeders + xxhash.c (tests/golden/make_ipt.py), and -- where
/root/reference is present -- agrees with that reference build on fresh random streams.
GPU: the host word-stream builder + batched device XXH64 (kbz_ipt_*) give the same keys, the
set novelty (kbz_set_*) the reference's HASH_FIND/HASH_ADD results in exec order, and the set's
state dump (insertion order) reloads into an identical set.
"""
import os

import numpy as np
import pytest

import oracle

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TAGS = ("libs", "nolibs")


def fixture():
    return np.load(os.path.join(G, "ipt.npz"), allow_pickle=False)


def libs_of(f, tag):
    libs = f["libs"] if tag == "libs" else f["libs"][:0]
    return libs[:, 0], libs[:, 1], libs[:, 2].astype(np.uint32)


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_matches_reference_fixture(oracle_lib, tag):
    f = fixture()
    keys = oracle.ipt_keys(f[f"{tag}_events"], *libs_of(f, tag), *f["target"].tolist())
    np.testing.assert_array_equal(keys, f[f"{tag}_keys"])


def test_oracle_matches_reference_build_random(oracle_lib):
    if not oracle.have_ref():
        pytest.skip("oracle/_ref not built (no /root/reference)")
    rng = np.random.default_rng(77)
    ev = []
    for _ in range(200):
        for _ in range(int(rng.integers(0, 30))):
            if rng.random() < 0.6:
                ev.append((0, int(rng.integers(0, 2**64, dtype=np.uint64)), int(rng.integers(0, 65))))
            else:
                ev.append((1, int(rng.integers(0, 2**64, dtype=np.uint64)), 0))
        ev.append((2, 0, 0))
    ev = np.array(ev, np.uint64)
    libs = (np.array([2**62], np.uint64), np.array([2**63], np.uint64), np.array([7], np.uint32))
    for lb in (libs, (libs[0][:0], libs[1][:0], libs[2][:0])):
        np.testing.assert_array_equal(oracle.ipt_keys(ev, *lb, 2**40, 2**41),
                                      oracle.ipt_keys(ev, *lb, 2**40, 2**41, use_ref=True))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_gpu_keys_and_novelty(gpu, tag):
    from killerbeez_amd.triage import IptBatch, UniqueSet

    f = fixture()
    starts, ends, hashes = libs_of(f, tag)
    b = IptBatch(list(zip(starts.tolist(), ends.tolist(), hashes.tolist())),
                 tuple(f["target"].tolist()))
    ev = f[f"{tag}_events"]
    ends_at = np.nonzero(ev[:, 0] == 2)[0]
    table = UniqueSet(4096)
    keys, isnew, lo = [], [], 0
    for cut in (ends_at[0], ends_at[99], ends_at[250], ends_at[-1]):  # uneven batches, carried set
        b.feed(ev[lo:cut + 1])
        k, nw = b.triage(table)
        keys.append(k)
        isnew.append(nw)
        lo = cut + 1
    np.testing.assert_array_equal(np.concatenate(keys), f[f"{tag}_keys"])
    np.testing.assert_array_equal(np.concatenate(isnew), f[f"{tag}_isnew"])
    # state dump (linux_ipt_get_state :986-1020: the keys in insertion order) and load
    # (linux_ipt_set_state :1040-1075: insert-if-absent in that order) give the same set
    dump = table.keys()
    assert dump.shape[0] == int(f[f"{tag}_isnew"].sum())
    np.testing.assert_array_equal(dump, f[f"{tag}_keys"][f[f"{tag}_isnew"] == 1])
    again = UniqueSet(4096)
    assert again.insert_host(dump).all()
    np.testing.assert_array_equal(again.keys(), dump)
    # device keys path (hash_device) equals the host path
    b.feed(ev)
    dk = b.hash_device().cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(dk, f[f"{tag}_keys"])
    b.close()


@pytest.mark.gpu
def test_gpu_long_streams(gpu):
    """Streams far longer than a 32-byte stripe (the 4-lane accumulator split) and empty ones."""
    from killerbeez_amd.triage import IptBatch

    rng = np.random.default_rng(9)
    ev = []
    for length in (0, 1, 3, 4, 5, 31, 32, 33, 1000, 20000):
        for _ in range(length):
            ev.append((0, int(rng.integers(0, 2**63)), 6))
            ev.append((1, int(rng.integers(0, 2**63)), 0))
        ev.append((2, 0, 0))
    ev = np.array(ev, np.uint64)
    b = IptBatch()
    b.feed(ev)
    got = b.hash_device().cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, oracle.ipt_keys(ev))
