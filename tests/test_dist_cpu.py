"""Multi-process (gloo, CPU) test of the sharded triage protocol in killerbeez_amd/dist.py.

The GPU engine (TriageContext) needs a GPU; here a CPU engine with the same shard_* methods,
built on the oracle (test infrastructure), runs the identical protocol: each rank triages its
contiguous shard, the ranks exchange last hashes and OR aggregates with all-gathers, and every
rank must end with exactly the per-trace results and virgin maps of one sequential pass over
the whole batch.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from killerbeez_amd import synth
from killerbeez_amd.dist import split_counts, timing_summary, triage_sharded

M = 4096


def _xform(mode, t, oc):
    t = t.copy()
    L = oracle.lib()
    for j in range(t.shape[0]):
        row = t[j]
        p = row.ctypes.data_as(oracle.C.c_void_p)
        if mode == oracle.MODE_DYNAMORIO:
            L.kbzo_classify_counts(p, M)
        elif oc[j] in (oracle.FUZZ_HANG, oracle.FUZZ_CRASH):
            L.kbzo_simplify_trace(p, M)
        elif mode == oracle.MODE_AFL_CLASSIFY:
            L.kbzo_classify_counts(p, M)
    return t


def _cls(mode, oc):
    if mode == oracle.MODE_DYNAMORIO:
        return np.zeros_like(oc, dtype=np.int64)
    return np.where(oc == oracle.FUZZ_HANG, 1, np.where(oc == oracle.FUZZ_CRASH, 2, 0))


class CpuShardEngine:
    """Oracle-backed stand-in for TriageContext's shard API (tests only)."""

    def __init__(self, mode, virgin, last_hash=0):
        self.mode = mode
        self.nc = 1 if mode == oracle.MODE_DYNAMORIO else 3
        self.map_size = M
        self.V = virgin.copy()
        self.last = last_hash

    def shard_begin(self, traces, outcome, want):
        self.t = traces.numpy()
        self.oc = outcome.numpy() if outcome is not None else np.zeros(self.t.shape[0], np.int8)
        self.x = _xform(self.mode, self.t, self.oc)
        self.h = np.array([oracle.hash32(r) for r in self.x], np.uint32)
        return {}

    def shard_last_row(self, out):
        if self.t.shape[0]:
            out.copy_(torch.from_numpy(self.t[-1]))

    def shard_last_hash(self, out):
        n = self.t.shape[0]
        out[0] = int(np.int32(np.uint32(self.h[-1] if n else 0).view(np.int32)))
        out[1] = 1 if n else 0

    def shard_link(self, prev_t, prev_row, is_first, glob_t, glob_row):
        n = self.t.shape[0]
        if not is_first:  # the previous shard's last row travels with its hash
            assert prev_row is not None and int(prev_t[1]) == 1
            assert oracle.hash32(_xform(self.mode, prev_row.numpy()[None], [0])[0]) == \
                np.uint32(np.int32(prev_t[0].item()))
        self.prev = self.last if is_first else int(np.uint32(np.int32(prev_t[0].item())))
        self.skip = np.zeros(n, bool)
        if self.mode == oracle.MODE_DYNAMORIO:
            for j in range(n):
                self.skip[j] = self.h[j] == (self.h[j - 1] if j else self.prev)
        self.next_last = int(np.uint32(np.int32(glob_t[0].item()))) if (
            glob_t is not None and int(glob_t[1])) else self.last

    def shard_reduce(self):
        cls = _cls(self.mode, self.oc)
        self.agg = np.zeros((self.nc, M), np.uint8)
        for j in range(self.t.shape[0]):
            if not self.skip[j]:
                self.agg[cls[j]] |= self.x[j]

    def shard_aggregate_bytes(self):
        return self.nc * M

    def shard_aggregate(self, out):
        out.copy_(torch.from_numpy(self.agg.reshape(-1)))

    @staticmethod
    def or_reduce(out, stacked, lo, hi, nb):
        out.copy_(torch.from_numpy(np.bitwise_or.reduce(stacked[lo:hi].numpy(), axis=0))
                  if hi > lo else torch.zeros(nb, dtype=torch.uint8))

    @staticmethod
    def or_prefix_total(prefix, total, stacked, rank, world, nb):
        """One pass over the gathered aggregates, as kbz_or_prefix_total does it."""
        acc = np.zeros(nb, np.uint8)
        rows = stacked.numpy()
        for r in range(world):
            if r == rank and prefix is not None:
                prefix.copy_(torch.from_numpy(acc.copy()))
            acc |= rows[r]
        total.copy_(torch.from_numpy(acc))
        # the fused pass equals the two separate reductions it replaces
        two = [torch.empty(nb, dtype=torch.uint8) for _ in range(2)]
        CpuShardEngine.or_reduce(two[0], stacked, 0, world, nb)
        CpuShardEngine.or_reduce(two[1], stacked, 0, rank, nb)
        assert torch.equal(two[0], total)
        assert prefix is None or torch.equal(two[1], prefix)

    def shard_finish(self, prefix, total):
        pre = np.zeros((self.nc, M), np.uint8) if prefix is None else prefix.numpy().reshape(self.nc, M)
        tot = total.numpy().reshape(self.nc, M)
        entry = self.V.copy()
        entry[:self.nc] &= ~pre
        r = oracle.triage_batch(self.mode, self.t, self.oc, virgin=entry, last_hash=self.prev)
        self.V[:self.nc] &= ~tot
        self.last = self.next_last
        return {"hnb": torch.from_numpy(r["hnb"])}


class CpuShardEngineFused(CpuShardEngine):
    """The fused-finish engine API (shard_exchange_row, shard_reduce_into,
    shard_finish_gathered: what TriageContext offers and dist.triage_sharded prefers), built
    from the steps it replaces -- so the gloo runs cover both protocol branches of dist.py."""

    def shard_exchange_row(self, out):
        self.shard_last_row(out[:M])
        self.shard_last_hash(out[M:M + 8].view(torch.int32))
        return out

    def shard_reduce_into(self, out):
        self.shard_reduce()
        return self.shard_aggregate(out)

    def shard_finish_gathered(self, gathered, rank, world):
        nb = self.shard_aggregate_bytes()
        total = torch.empty(nb, dtype=torch.uint8)
        prefix = torch.empty(nb, dtype=torch.uint8) if rank > 0 else None
        self.or_prefix_total(prefix, total, gathered, rank, world, nb)
        return self.shard_finish(prefix, total)


def _worker(rank, world, port, mode, counts, seed, q, fused=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t, oc = synth.sparse_np(sum(counts), M, seed=seed, hot_frac=0.05)
    t[40] = t[39]  # DynamoRIO skip inside / across shards
    if sum(counts) > 51:
        t[51] = t[50]
    lo = sum(counts[:rank])
    eng = (CpuShardEngineFused if fused else CpuShardEngine)(mode, np.full((3, M), 0xFF, np.uint8))
    hnbs, timings = [], []
    for batch in range(2):  # two consecutive sharded batches: state carries over
        tt = t if batch == 0 else t[::-1].copy()
        oo = oc if batch == 0 else oc[::-1].copy()
        mine = torch.from_numpy(tt[lo:lo + counts[rank]].copy())
        out = triage_sharded(eng, mine, torch.from_numpy(oo[lo:lo + counts[rank]].copy()),
                             counts, rank, world, device="cpu", timings=timings)
        hnbs.append(out["hnb"].numpy())
    ph = timing_summary(timings)
    assert {"pass1", "reduce", "collective", "finish"} <= set(ph), ph
    q.put((rank, hnbs, eng.V, eng.last))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("fused", [False, True], ids=["staged", "fused-finish"])
@pytest.mark.parametrize("mode", [oracle.MODE_AFL, oracle.MODE_DYNAMORIO])
@pytest.mark.parametrize("counts", [[60, 40], [50, 0, 47]])
def test_sharded_equals_sequential(oracle_lib, mode, counts, fused):
    world = len(counts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, counts, 7, q, fused))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, hnbs, V, last = q.get(timeout=300)
        res[r] = (hnbs, V, last)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # sequential reference over the whole batch, twice
    t, oc = synth.sparse_np(sum(counts), M, seed=7, hot_frac=0.05)
    t[40] = t[39]
    if sum(counts) > 51:
        t[51] = t[50]
    V = np.full((3, M), 0xFF, np.uint8)
    last = 0
    for batch in range(2):
        tt = t if batch == 0 else t[::-1].copy()
        oo = oc if batch == 0 else oc[::-1].copy()
        r = oracle.triage_batch(mode, tt, oo, virgin=V, last_hash=last)
        V, last = r["virgin"], r["last_hash"]
        got = np.concatenate([res[k][0][batch] for k in range(world)])
        np.testing.assert_array_equal(got, r["hnb"])
    for k in range(world):
        np.testing.assert_array_equal(res[k][1], V)
        if mode == oracle.MODE_DYNAMORIO:
            assert res[k][2] == last
