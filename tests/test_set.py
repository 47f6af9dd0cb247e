"""The unique crash/hang table (kbz_set_*): insert-if-absent over an ordered batch.

Expected values come from a plain insertion-ordered dict, the semantics of the reference's
uthash set at linux_ipt_instrumentation.c:412-424 (HASH_FIND; HASH_ADD when absent; "new" iff
absent; iteration in insertion order).  This is a new feature on the path (XXH64 keys of
crash/hang maps, BASELINE config 5): parity is anchored on that call site's semantics and on the
XXH64 values, which are pinned to the reference's xxHash (tests/test_oracle_pin.py).
"""
import numpy as np
import pytest

import oracle
from killerbeez_amd import synth


def reference_set(batches, masks=None):
    seen = {}
    out = []
    for b, keys in enumerate(batches):
        new = np.zeros(len(keys), np.uint8)
        for j, k in enumerate(map(tuple, keys)):
            if masks is not None and not masks[b][j]:
                continue
            if k not in seen:  # HASH_FIND miss -> HASH_ADD
                seen[k] = len(seen)
                new[j] = 1
        out.append(new)
    return out, np.array(list(seen.keys()), np.uint64).reshape(-1, 2)


def test_reference_set_semantics():
    out, keys = reference_set([np.array([[1, 2], [1, 2], [3, 4]], np.uint64),
                               np.array([[3, 4], [5, 6]], np.uint64)])
    assert out[0].tolist() == [1, 0, 1] and out[1].tolist() == [0, 1]
    assert keys.tolist() == [[1, 2], [3, 4], [5, 6]]


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


@pytest.mark.gpu
def test_insert_batches_with_repeats_and_collisions(gpu):
    from killerbeez_amd.triage import UniqueSet

    rng = np.random.default_rng(1)
    pool = rng.integers(0, 2**63, size=(300, 2), dtype=np.uint64)
    pool[5, 0] = pool[6, 0]          # same low word, different high word
    pool[7] = [2**64 - 1, 2**64 - 1]  # all-ones key (the table's empty marker value)
    batches, masks = [], []
    for b in range(5):
        idx = rng.integers(0, 300, size=800)
        batches.append(pool[idx])
        masks.append(rng.random(800) < 0.9)
    exp, exp_keys = reference_set(batches, masks)
    s = UniqueSet(4096)
    import torch

    for b in range(5):
        got = s.insert(_dev(batches[b]), torch.from_numpy(masks[b]).cuda()).cpu().numpy()
        np.testing.assert_array_equal(got, exp[b])
    assert s.size() == len(exp_keys)
    np.testing.assert_array_equal(s.keys(), exp_keys)


@pytest.mark.gpu
def test_capacity_exceeded_is_an_error(gpu):
    from killerbeez_amd._lib import KbzError
    from killerbeez_amd.triage import UniqueSet

    s = UniqueSet(4)  # 16 slots
    keys = np.arange(80, dtype=np.uint64).reshape(40, 2)
    s.insert(_dev(keys))
    with pytest.raises(KbzError, match="capacity"):
        s.size()


@pytest.mark.gpu
def test_unique_crashes_from_triage(gpu):
    """Config 5's table: XXH64 of each crash/hang trace's simplified map + its class; a trace is
    a unique crash/hang iff its key is new."""
    import torch

    from killerbeez_amd.triage import MODE_AFL, WANT_H32, WANT_X64, TriageContext, UniqueSet, \
        dedup_keys

    t, oc = synth.sparse_np(600, 4096, seed=31, hot_frac=0.01, outcome_p=(0.6, 0.2, 0.2))
    t[100:140] = t[99]                     # a crash repeated many times
    oc[99:140] = 2
    exp = oracle.triage_batch(MODE_AFL, t, oc, want=oracle.WANT_H32 | oracle.WANT_X64)
    keys = np.stack([exp["x64"], oc.astype(np.uint64)], axis=1)
    mask = oc != 0
    exp_new, _ = reference_set([keys], [mask])
    with TriageContext(4096, MODE_AFL, 600) as ctx:
        to = torch.from_numpy(oc).cuda()
        out = ctx.triage(torch.from_numpy(t).cuda(), to, WANT_H32 | WANT_X64)
        s = UniqueSet(1024)
        got = s.insert(dedup_keys(out["x64"], to), to != 0).cpu().numpy()
    np.testing.assert_array_equal(got, exp_new[0])
    assert got[99] == 1 and not got[100:140].any()


def reference_merge(first_keys, second_keys):
    """linux_ipt_merge (linux_ipt_instrumentation.c:944-978): a fresh table, every entry of the
    first state (HASH_ITER order = insertion order), then each entry of the second state that
    HASH_FIND misses."""
    seen = {}
    for k in map(tuple, first_keys):
        seen.setdefault(k, len(seen))
    for k in map(tuple, second_keys):
        if k not in seen:
            seen[k] = len(seen)
    return np.array(list(seen.keys()), np.uint64).reshape(-1, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("n_a,n_b", [(700, 900), (0, 300), (300, 0), (1, 1)])
def test_merge_like_linux_ipt_merge(gpu, n_a, n_b):
    from killerbeez_amd.triage import UniqueSet

    rng = np.random.default_rng(n_a * 7 + n_b)
    pool = rng.integers(0, 2**63, size=(500, 2), dtype=np.uint64)
    pool[3, 0] = pool[4, 0]  # same low word, different high word
    a_rows = pool[rng.integers(0, 500, size=n_a)]
    b_rows = pool[rng.integers(0, 500, size=n_b)]
    a, b = UniqueSet(1024), UniqueSet(2048)
    if n_a:
        a.insert(_dev(a_rows))
    if n_b:
        b.insert(_dev(b_rows))
    a_keys, b_keys = a.keys(), b.keys()
    m = a.merge(b)
    exp = reference_merge(a_keys, b_keys)
    assert m.size() == len(exp)
    np.testing.assert_array_equal(m.keys(), exp)
    # inputs unchanged; the merged set keeps answering novelty like the reference's table
    np.testing.assert_array_equal(a.keys(), a_keys)
    np.testing.assert_array_equal(b.keys(), b_keys)
    probe = np.concatenate([pool[:50], rng.integers(0, 2**63, size=(20, 2), dtype=np.uint64)])
    got = m.insert(_dev(probe)).cpu().numpy()
    exp_new, _ = reference_set([np.concatenate([exp, probe])])
    np.testing.assert_array_equal(got, exp_new[0][len(exp):])
