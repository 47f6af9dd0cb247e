#!/usr/bin/env python3
"""Headline benchmark: traces triaged/s (64 KiB map, classify + novelty + hash32) on MI355X.

Workload (BASELINE.json configs[1]): per GPU a batch of 65,536
synthetic sparse traces x 64 KiB raw hit counters (seeded generator in killerbeez_amd.synth,
generated directly in HBM), triaged with DynamoRIO semantics (dynamorio_instrumentation.c:
1428-1468: classify_counts, hash32, last-hash skip, has_new_bits vs virgin_bits).  One step =
one full triage of one batch; the virgin map and last hash carry over from step to step
(steady-state fuzzing), cycling through a pool of distinct batches.

With --gpus N (launched by torch.distributed.run) every rank triages its own 65,536-trace
shard of an N x 65,536-trace global batch with the exact sharded protocol of
killerbeez_amd.dist (RCCL all-gathers) -- weak scaling.

Prints ONE JSON line (rank 0).  Also reports the dominant kernel's (pass 1) achieved
algorithmic HBM bandwidth against the 8 TB/s peak, and the reference CPU path timed on this
host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "traces triaged/sec (64KB map, classify+novelty+hash) and % HBM peak, 1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=65536, help="traces per GPU per step")
    p.add_argument("--map-size", type=int, default=65536)
    p.add_argument("--mode", default="dynamorio", choices=["dynamorio", "afl", "afl_classify"])
    p.add_argument("--pool", type=int, default=2, help="distinct batches cycled through")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--seed", type=int, default=0x5EED)
    return p.parse_args()


def cpu_baseline(traces_dev, mode, seconds):
    """Reference CPU path (oracle/_ref: the reference's own classify_counts + hash32 +
    has_new_bits in has_new_coverage's control flow), one core, on a bounded sample of the
    same workload.  Falls back to the clean-room restatement if _ref is absent."""
    import ctypes as C

    import numpy as np

    import oracle

    m = traces_dev.shape[1]
    sample_n = min(traces_dev.shape[0], 8192)
    host = traces_dev[:sample_n].cpu().numpy()
    virgin = np.full(m, 0xFF, np.uint8)
    scratch = np.empty(m, np.uint8)
    hnb = np.zeros(sample_n, np.uint8)
    last = C.c_uint32(0)
    sfx = {65536: "64k", 1 << 20: "1m"}.get(m)
    kind = "reference"
    fn = None
    if mode == 1 and sfx and oracle.have_ref():
        fn = getattr(oracle.ref(), f"ref_dr_triage_loop_{sfx}")
        fn.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                       C.c_void_p]
    done, t0 = 0, time.perf_counter()
    passes = 0
    while True:
        if fn is not None:
            fn(host.ctypes.data_as(C.c_void_p), sample_n, m, virgin.ctypes.data_as(C.c_void_p),
               C.byref(last), hnb.ctypes.data_as(C.c_void_p), scratch.ctypes.data_as(C.c_void_p))
        else:
            kind = "port"
            oracle.triage_batch(mode, host, None, threads=0)
        done += sample_n
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "traces/s", "cores": 1, "kind": kind,
            "sample": f"{sample_n} traces x {m} B of the bench workload, {passes} sequential "
                      f"passes ({el:.1f} s), virgin carried, 1 thread"}


def cpu_baseline_all_cores(traces_dev, mode, seconds):
    """Clean-room restatement, exact sharded decomposition over all host cores (port)."""
    import numpy as np

    import oracle

    threads = min(os.cpu_count() or 1, 16)  # the GPU box's CPU share is 16 threads
    sample_n = min(traces_dev.shape[0], 8192)
    host = traces_dev[:sample_n].cpu().numpy()
    done, t0 = 0, time.perf_counter()
    while True:
        oracle.triage_batch(mode, host, None, threads=threads)
        done += sample_n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "traces/s", "cores": threads, "kind": "port",
            "sample": f"{sample_n} traces, oracle/kbz_oracle.c kbzo_triage_batch_mt"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from killerbeez_amd import synth
    from killerbeez_amd.dist import triage_sharded
    from killerbeez_amd.triage import MODES, WANT_H32, TriageContext

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    mode = MODES[args.mode]
    B, M = args.batch, args.map_size

    pool = []
    for p in range(args.pool):
        t, oc = synth.sparse_torch(B, M, seed=args.seed + 7919 * p + 104729 * rank, device=dev)
        pool.append((t, oc))
    ctx = TriageContext(M, mode, B)
    out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev),
           "h32": torch.empty(B, dtype=torch.int32, device=dev)}
    counts = [B] * world

    timings = []

    def step(i, record=False):
        t, oc = pool[i % len(pool)]
        ctx._out = out
        if world == 1:
            ev = None
            if record:
                ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
                ev[0].record()
            ctx.shard_begin(t, oc, WANT_H32, out=out)
            if record:
                ev[1].record()
                timings.append(ev)
            ctx.shard_link(None, True, None)
            ctx.shard_reduce()
            ctx.shard_finish(None, _total(ctx))
        else:
            ctx_out = triage_sharded(ctx, t, oc, counts, rank, world, WANT_H32, device=dev,
                                     timings=timings if record else None)
            del ctx_out

    agg_buf = {}

    def _total(c):
        nb = c.shard_aggregate_bytes()
        if nb not in agg_buf:
            agg_buf[nb] = torch.empty(nb, dtype=torch.uint8, device=dev)
        c.shard_aggregate(agg_buf[nb])
        return agg_buf[nb]

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    ctx.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, record=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    ctx.sync()
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    pass1_ms = sum(a.elapsed_time(b) for a, b in timings) / max(1, len(timings))
    total_traces = world * B * args.steps
    value = total_traces / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    achieved = B * M / (pass1_ms * 1e-3) / 1e9  # GB/s, algorithmic bytes of one launch
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pass1_traffic.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    res = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "traces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY.md §8(d) config 2 generator, seeded, generated in HBM)",
        "config": {"workload": f"config2: {B} sparse traces/GPU x {M} B map, {args.mode} "
                               "classify+hash32+last-hash skip+has_new_bits, virgin carried",
                   "map_size": M, "batch_per_gpu": B, "global_batch": world * B,
                   "mode": args.mode, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": "k_pass1 (+2 tiny memsets)",
                     "avg_launch_ms": round(pass1_ms, 4),
                     "algorithmic_bytes_per_launch": B * M},
        "pass1_share_of_step": round(pass1_ms / ms_per_step, 4),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(pool[0][0], mode, args.cpu_seconds)
        res["cpu_baseline_all_cores"] = cpu_baseline_all_cores(pool[0][0], mode,
                                                               max(2.0, args.cpu_seconds / 3))
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
