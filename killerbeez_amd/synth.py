"""Seeded synthetic trace batches.

sparse (config 2): a hot edge set of round(hot_frac*map_size) random positions; every trace
    hits each hot edge with probability p_hot, count ~ Geometric(geo_p) capped at 255; plus
    Poisson(cold_rate) cold edges uniform over the map with counts U[1,255]; outcome NONE /
    HANG / CRASH with probabilities (0.98, 0.005, 0.015).
dense (config 3): hot_frac 0.5 and counts U[1,255].
uniform: every byte nonzero with probability `density`, counts U[1,255].

Counts are raw 8-bit hit counters as the instrumented target writes them
(afl_progs/afl-as.h:426-443: map[cur ^ prev]++ with 8-bit wrap).
"""
from __future__ import annotations

import math

import numpy as np

OUTCOME_P = (0.98, 0.005, 0.015)  # NONE, HANG, CRASH


def _counts_np(rng, shape, geo_p, uniform_counts):
    if uniform_counts:
        return rng.integers(1, 256, size=shape, dtype=np.int64)
    return np.minimum(rng.geometric(geo_p, size=shape), 255)


def sparse_np(n, map_size=65536, seed=0x5EED, hot_frac=0.02, p_hot=0.9, geo_p=0.35,
              cold_rate=0.5, uniform_counts=False, outcome_p=OUTCOME_P):
    """numpy generator (tests / CPU baseline).  Returns (traces uint8 [n, M], outcome int8)."""
    rng = np.random.default_rng(seed)
    H = max(1, int(round(hot_frac * map_size)))
    hot = rng.permutation(map_size)[:H]
    t = np.zeros((n, map_size), np.uint8)
    if n == 0:
        return t, np.zeros(0, np.int8)
    inc = rng.random((n, H)) < p_hot
    cnt = _counts_np(rng, (n, H), geo_p, uniform_counts)
    t[:, hot] = np.where(inc, cnt, 0).astype(np.uint8)
    k = rng.poisson(cold_rate, size=n)
    tot = int(k.sum())
    if tot:
        rows = np.repeat(np.arange(n), k)
        cols = rng.integers(0, map_size, size=tot)
        t[rows, cols] = rng.integers(1, 256, size=tot).astype(np.uint8)
    oc = rng.choice(3, size=n, p=outcome_p).astype(np.int8)
    return t, oc


def dense_np(n, map_size=1 << 20, seed=0x5EED, **kw):
    kw.setdefault("hot_frac", 0.5)
    kw.setdefault("uniform_counts", True)
    kw.setdefault("cold_rate", 0.0)
    return sparse_np(n, map_size, seed, **kw)


def uniform_np(n, map_size=65536, seed=0, density=0.02):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, map_size)) < density
    vals = rng.integers(1, 256, size=(n, map_size), dtype=np.uint8)
    return np.where(mask, vals, 0).astype(np.uint8)


def sparse_torch(n, map_size=65536, seed=0x5EED, device="cuda", hot_frac=0.02, p_hot=0.9,
                 geo_p=0.35, cold_rate=0.5, uniform_counts=False, outcome_p=OUTCOME_P,
                 out=None, block=4096, hot_seed=None):
    """Same distribution generated directly in device memory (bench inputs, HBM-resident).
    hot_seed: seed of the hot edge set alone (batches of one target program share it; default:
    drawn from `seed`).  Returns (traces uint8 [n, M] on device, outcome int8 [n] on device)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    H = max(1, int(round(hot_frac * map_size)))
    if hot_seed is None:
        hot = torch.randperm(map_size, generator=g, device=device)[:H]
    else:
        gh = torch.Generator(device=device)
        gh.manual_seed(hot_seed)
        hot = torch.randperm(map_size, generator=gh, device=device)[:H]
    t = out if out is not None else torch.empty((n, map_size), dtype=torch.uint8, device=device)
    t.zero_()
    lg = math.log1p(-geo_p)
    for lo in range(0, n, block):
        b = min(block, n - lo)
        inc = torch.rand((b, H), generator=g, device=device) < p_hot
        if uniform_counts:
            cnt = torch.randint(1, 256, (b, H), generator=g, device=device)
        else:
            u = torch.rand((b, H), generator=g, device=device).clamp_min_(1e-12)
            cnt = (torch.floor(torch.log(u) / lg) + 1).clamp_(1, 255)
        vals = torch.where(inc, cnt, torch.zeros_like(cnt)).to(torch.uint8)
        t[lo:lo + b].index_copy_(1, hot, vals)
        if cold_rate > 0:
            k = torch.poisson(torch.full((b,), float(cold_rate), device=device), generator=g)
            k = k.to(torch.int64)
            tot = int(k.sum().item())
            if tot:
                rows = torch.repeat_interleave(torch.arange(b, device=device), k) + lo
                cols = torch.randint(0, map_size, (tot,), generator=g, device=device)
                v = torch.randint(1, 256, (tot,), generator=g, device=device).to(torch.uint8)
                t[rows, cols] = v
    p = torch.tensor(outcome_p, device=device, dtype=torch.float64).cumsum(0)
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    oc = torch.searchsorted(p, u).clamp_(0, 2).to(torch.int8)
    return t, oc


def dense_torch(n, map_size=1 << 20, seed=0x5EED, device="cuda", **kw):
    kw.setdefault("hot_frac", 0.5)
    kw.setdefault("uniform_counts", True)
    kw.setdefault("cold_rate", 0.0)
    return sparse_torch(n, map_size, seed, device, **kw)


def merger_states_np(n_states, map_size=65536, seed=0, clear_p=0.02):
    """Merger config 4: each state = 3 all-0xff maps with a Bernoulli(clear_p) random subset
    of bits cleared."""
    rng = np.random.default_rng(seed)
    s = np.full((n_states, 3 * map_size), 0xFF, np.uint8)
    bits = rng.random((n_states, 3 * map_size, 8)) < clear_p
    clear = np.packbits(bits, axis=-1, bitorder="little")[..., 0]
    return s & ~clear


def with_repeats_torch(traces, outcome, frac=0.9, seed=0):
    """In place: every exec after the first repeats its predecessor (same trace, same outcome)
    with probability `frac` -- the runs of identical execs of real fuzzing, where most mutations
    do not change the path (the DynamoRIO last-hash skip's workload).  Returns the number of
    repeated rows."""
    import torch

    n = traces.shape[0]
    if n < 2:
        return 0
    g = torch.Generator(device=traces.device)
    g.manual_seed(seed)
    rep = torch.rand(n, generator=g, device=traces.device) < frac
    rep[0] = False
    idx = torch.arange(n, device=traces.device)
    src = torch.cummax(torch.where(rep, torch.zeros_like(idx), idx), 0).values
    traces.copy_(traces[src])
    outcome.copy_(outcome[src])
    return int(rep.sum().item())
