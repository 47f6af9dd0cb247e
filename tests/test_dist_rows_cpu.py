"""Multi-process (gloo, CPU) tests of the two other sharded rows of SURVEY.md §8(e):

* merge_sharded -- the merger fold across ranks (local AND-fold, all-gather of the partial
  folds, local AND) must equal the sequential fold merger/merger.c:79-99 performs;
* dedup_sharded -- the unique crash/hang table across ranks (all-gather of the masked keys in
  rank = global order, ordered insert into every rank's replica) must equal one insert-if-absent
  pass over the whole batch in trace order (linux_ipt_instrumentation.c:412-424), with every
  replica holding the same keys in the same insertion order.

The GPU fold / table are replaced by CPU stand-ins with the same interface (the oracle's
restated merge_bitmaps loop; an insertion-ordered dict), so the protocol itself runs here.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from killerbeez_amd.dist import dedup_sharded, merge_sharded, split_counts

SB = 3 * 4096


def _fold(rows, out=None):
    r = rows.numpy()
    res = torch.from_numpy(oracle.merge_many(r).reshape(-1) if r.shape[0]
                           else np.full(r.shape[1], 0xFF, np.uint8))
    if out is not None:
        out.copy_(res)
        return out
    return res


class OrderedSetTable:
    """Stand-in for UniqueSet: insert-if-absent, insertion order kept (uthash HASH_ADD)."""

    def __init__(self):
        self.keys = {}

    def insert(self, keys, mask=None):
        out = torch.zeros(keys.shape[0], dtype=torch.uint8)
        m = [1] * keys.shape[0] if mask is None else mask.tolist()
        for j, (a, b) in enumerate(keys.tolist()):
            if m[j] and (a, b) not in self.keys:
                self.keys[(a, b)] = len(self.keys)
                out[j] = 1
        return out


def _states(n, seed):
    rng = np.random.default_rng(seed)
    s = np.full((n, SB), 0xFF, np.uint8)
    pos = rng.integers(0, n * SB * 8, size=SB * 4)
    np.bitwise_and.at(s.reshape(-1), pos // 8, ~(np.uint8(1) << (pos % 8).astype(np.uint8)))
    return s


def _keys(n, seed):
    rng = np.random.default_rng(seed)
    k = np.stack([rng.integers(0, 40, n), rng.integers(1, 3, n)], axis=1).astype(np.int64)
    mask = rng.random(n) < 0.6
    return k, mask


def _worker(rank, world, port, counts, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, n = sum(counts[:rank]), counts[rank]
    s = _states(sum(counts), 11)
    merged = merge_sharded(torch.from_numpy(s[lo:lo + n].copy()).view(n, SB), world, fold=_fold)
    tab = OrderedSetTable()
    news = []
    for b in range(3):  # three batches: the replica carries over; the last one without a cap
        k, m = _keys(sum(counts), 20 + b)   # (the ranks negotiate it: unequal shards)
        news.append(dedup_sharded(tab, torch.from_numpy(k[lo:lo + n].copy()),
                                  torch.from_numpy(m[lo:lo + n].copy()), rank, world,
                                  cap=max(counts) if b < 2 else None).numpy())
    q.put((rank, merged.numpy(), news, list(tab.keys)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("counts", [[90, 70], [50, 0, 47], split_counts(101, 3)])
def test_merge_and_dedup_sharded(oracle_lib, counts):
    world = len(counts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, merged, news, keys = q.get(timeout=300)
        res[r] = (merged, news, keys)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = sum(counts)
    # merger: the sequential fold of all states (merger.c:79-99 over the reference's merge_bitmaps)
    s = _states(n, 11)
    exp = np.full(SB, 0xFF, np.uint8)
    for i in range(n):
        exp &= s[i]
    # dedup: one insert-if-absent pass in global trace order
    seen, exp_new = {}, []
    for b in range(3):
        k, m = _keys(n, 20 + b)
        e = np.zeros(n, np.uint8)
        for j in range(n):
            key = tuple(int(x) for x in k[j])
            if m[j] and key not in seen:
                seen[key] = len(seen)
                e[j] = 1
        exp_new.append(e)
    for r in range(world):
        np.testing.assert_array_equal(res[r][0], exp)
        assert res[r][2] == list(seen)  # same keys, same insertion order, on every replica
    for b in range(3):
        got = np.concatenate([res[r][1][b] for r in range(world)])
        np.testing.assert_array_equal(got, exp_new[b])
