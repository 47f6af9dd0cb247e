"""Multi-GPU sharded triage: one process per GPU, torch.distributed (RCCL over xGMI).

A batch of N traces is split into contiguous shards, rank g holding [lo_g, hi_g).  Order is
preserved, so the reference's sequential semantics hold across shards once every rank knows
the OR of the coverage seen by the ranks before it:

  1. local pass over the shard (kbz_shard_begin: hashes, chunk aggregates)   -- no traffic
  2. DynamoRIO only: one all-gather of each shard's last hash32 and last raw trace (8 B +
     map_size per rank); the first trace of a shard is compared with the last trace of the
     nearest non-empty earlier shard (hash for the skip rule, row for its exactness), and every
     rank remembers the batch's last row for the next batch
  3. local OR aggregate per virgin map (kbz_shard_reduce_into: straight into the buffer the
     all-gather sends)
  4. all-gather of the aggregates (nclass * map_size bytes per rank) -> prefix = OR of earlier
     ranks, total = OR of all ranks.  RCCL has no bitwise reductions, so this is an
     all-gather; the OR of the gathered rows happens inside the resolve (~8 x 64 KiB over xGMI:
     latency-bound).
  5. local resolve with the prefix (kbz_shard_finish_gathered: the one-shard batch's fused tail,
     k_tail + k_fin); every rank applies V' = V & ~total, so the virgin maps stay identical on
     all ranks.
Engines without the fused finish (the tests' CPU engine) run the same steps with separate
aggregate copy, prefix / total pass and finish (kbz_shard_reduce, kbz_or_prefix_total,
kbz_shard_finish).

The engine is any object with the shard_* methods of killerbeez_amd.triage.TriageContext
(tests plug a CPU engine in to exercise this protocol with the gloo backend).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

MODE_DYNAMORIO = 1


def split_counts(n_total: int, world: int) -> list[int]:
    return [n_total * (r + 1) // world - n_total * r // world for r in range(world)]


def _all_gather(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """[world, *t.shape]: one all_gather_into_tensor into a flat buffer (no per-rank list, no
    stack; gloo accepts only the flat output shape)."""
    t = t.contiguous()
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.reshape(-1), group=group)
    return out.view(world, *t.shape)


class _Clock:
    """Phase timing of one rank's sharded batch: HIP events on the current stream when the
    tensors live on a GPU (read after the batch), wall clock otherwise."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.marks = []

    def mark(self, name):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))

    def spans(self):
        """{phase: ms} between consecutive marks (phase = the later mark's name)."""
        out = {}
        for (_, a), (name, b) in zip(self.marks, self.marks[1:]):
            ms = a.elapsed_time(b) if self.cuda else 1e3 * (b - a)
            out[name] = out.get(name, 0.0) + ms
        return out


def triage_sharded(engine, traces, outcome, counts, rank, world, want=1, group=None,
                   device=None, timings=None, force_collective=False):
    """Run one rank's part of a sharded batch.  counts[r] = number of traces on rank r (host
    ints, known to every rank).  Returns the engine's output dict (hnb, h32, ...).
    timings: a list that receives this batch's phase times {pass1, link, reduce, collective,
    finish} in ms (HIP events on a GPU, read with timing_summary after the steps).
    force_collective: run the all-gathers even at world 1 (a one-rank RCCL communicator
    exercises the exchange path on a one-GPU box)."""
    coll = world > 1 or force_collective
    device = device if device is not None else traces.device
    clk = _Clock(device) if timings is not None else None
    mark = clk.mark if clk else (lambda name: None)
    # engines with the fused finish (TriageContext): one launch for the link exchange, the
    # aggregate written into its all-gather slot, prefix / total taken inside the fused tail
    fused = hasattr(engine, "shard_finish_gathered")
    mark("start")
    out = engine.shard_begin(traces, outcome, want)
    mark("pass1")
    nonempty = [r for r in range(world) if counts[r] > 0]
    if engine.mode == MODE_DYNAMORIO:
        m = engine.map_size
        # [last row | hash pair | pad]: map_size + 16 bytes, so every gathered row stays
        # 16-byte aligned (k_chain reads rows with 16-byte loads)
        buf = torch.zeros(m + 16, dtype=torch.uint8, device=device)
        if fused:
            engine.shard_exchange_row(buf)
        else:
            engine.shard_last_row(buf[:m])
            engine.shard_last_hash(buf[m:m + 8].view(torch.int32))
        mark("link")
        bufs = _all_gather(buf, world, group) if coll else buf.view(1, -1)
        mark("collective")
        rows, pairs = bufs[:, :m], bufs[:, m:m + 8].view(torch.int32)
        prev = [r for r in nonempty if r < rank]
        p = prev[-1] if prev else None
        g = nonempty[-1] if nonempty else None
        engine.shard_link(None if p is None else pairs[p], None if p is None else rows[p],
                          not prev, None if g is None else pairs[g],
                          None if g is None else rows[g])
    else:
        engine.shard_link(None, None, True, None, None)
    mark("link")
    nb = engine.shard_aggregate_bytes()
    if fused:
        agg = torch.empty(nb, dtype=torch.uint8, device=device)
        engine.shard_reduce_into(agg)
        mark("reduce")
        allagg = _all_gather(agg, world, group) if coll else agg.view(1, nb)
        if coll:
            mark("collective")
        res = engine.shard_finish_gathered(allagg, rank if coll else 0, world if coll else 1)
        mark("finish")
        if clk is not None:
            timings.append(clk)
        return res
    engine.shard_reduce()
    agg = torch.empty(nb, dtype=torch.uint8, device=device)
    engine.shard_aggregate(agg)
    mark("reduce")
    if coll:
        allagg = _all_gather(agg, world, group)
        mark("collective")
        total = torch.empty(nb, dtype=torch.uint8, device=device)
        prefix = torch.empty(nb, dtype=torch.uint8, device=device) if rank > 0 else None
        engine.or_prefix_total(prefix, total, allagg, rank, world, nb)
    else:
        total, prefix = agg, None
    res = engine.shard_finish(prefix, total)
    mark("finish")
    if clk is not None:
        timings.append(clk)
    return res


def timing_summary(timings):
    """Mean ms per batch of each phase over the recorded batches (waits for their events)."""
    if not timings:
        return {}
    if timings[0].cuda:
        torch.cuda.synchronize()
    tot = {}
    for clk in timings:
        for k, v in clk.spans().items():
            tot[k] = tot.get(k, 0.0) + v
    return {k: v / len(timings) for k, v in tot.items()}


# ---- merger across GPUs (BASELINE config 4) ----------------------------------

def merge_sharded(states, world, group=None, fold=None, out=None, force_collective=False):
    """The merger's AND-fold (merger/merger.c:79-99 -> afl_merge afl_instrumentation.c:123-140)
    over states spread across ranks: every rank folds its own states (rows of `states`, any
    count, possibly 0) with one local AND-fold, the ranks all-gather their partial folds
    (state_bytes each, over xGMI), and every rank ANDs the world partials.  AND is associative
    and commutative, so the result equals the sequential fold of all states in any order.
    `fold(rows, out=None)` is the local AND-fold (default: kbz_merge_and_device); RCCL has no
    bitwise-AND reduction, hence all-gather + local fold.  Returns the merged state (every
    rank holds it).  force_collective: all-gather even at world 1."""
    if fold is None:
        from .triage import merge_and as fold
    local = fold(states)
    if world == 1 and not force_collective:
        if out is not None:
            out.copy_(local)
            return out
        return local
    parts = _all_gather(local.contiguous(), world, group)
    return fold(parts, out=out)


# ---- unique crash/hang table across GPUs (BASELINE config 5) ----------------

def dedup_sharded(table, keys, mask, rank, world, group=None, cap=None, force_collective=False):
    """The reference's insert-if-absent set novelty (linux_ipt_instrumentation.c:412-424: new iff
    the key was absent; HASH_ADD keeps insertion order) over a batch sharded by contiguous trace
    index.  keys: this rank's [n_r, 2] int64 keys (e.g. {XXH64 of the transformed trace,
    outcome class}: triage.dedup_keys); mask: [n_r] bool/uint8, rows that take part (crash and
    hang traces).  Every rank's rows are all-gathered in rank order -- i.e. in global trace
    order -- as ONE fixed-shape buffer of cap rows per rank {key, mask} (padding rows masked
    out; cap = the largest shard), and inserted as one ordered, masked batch into every rank's
    replica `table` (any object with UniqueSet.insert(keys, mask)), so all replicas stay
    identical and the first occurrence in global order is the new one.  With `cap` given there
    is no host synchronisation and no host-side concatenation (the masking happens in the
    insert); without it, one all_reduce(MAX) of the shard sizes finds it (one host sync), so
    unequal shards are always handled.  Returns this rank's is_new [n_r] uint8 (0 for masked-out
    rows).  force_collective: all-gather even at world 1."""
    dev = keys.device
    n = keys.shape[0]
    m8 = mask.to(torch.int64).view(-1, 1)
    if world == 1 and not force_collective:
        return table.insert(keys, mask=mask.to(torch.uint8)).to(torch.uint8)
    if cap is None:
        c = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
        cap = int(c.item())
    if n > cap:
        raise ValueError("dedup_sharded: shard larger than cap")
    buf = torch.zeros((cap, 3), dtype=torch.int64, device=dev)
    buf[:n, :2] = keys
    buf[:n, 2:] = m8
    allb = _all_gather(buf, world, group).view(world * cap, 3)
    isnew = table.insert(allb[:, :2].contiguous(), mask=allb[:, 2].to(torch.uint8))
    return isnew[rank * cap:rank * cap + n].to(torch.uint8)
