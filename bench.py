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
    p.add_argument("--workload", default="config2",
                   choices=["config2", "config3", "merge", "stream"],
                   help="config2 (default, the headline): 65,536 sparse x 64 KiB; config3: "
                        "16,384 dense x 1 MiB; merge: 100k merger states AND-folded; stream: "
                        "config2 traces from host memory through the pinned ring (PCIe-bound)")
    p.add_argument("--states", type=int, default=100000, help="merge workload: states")
    a = p.parse_args()
    if a.workload == "config3":
        if a.batch == 65536:
            a.batch = 16384
        if a.map_size == 65536:
            a.map_size = 1 << 20
    return a


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
    if args.workload == "merge":
        return main_merge(args)
    if args.workload == "stream":
        return main_stream(args)
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
    gen = synth.dense_torch if args.workload == "config3" else synth.sparse_torch
    for p in range(args.pool):
        t, oc = gen(B, M, seed=args.seed + 7919 * p + 104729 * rank, device=dev)
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
            ctx.shard_link(None, None, True, None, None)
            ctx.shard_reduce()
            ctx.shard_finish(None, None)  # single shard: its own aggregate is the total
        else:
            ctx_out = triage_sharded(ctx, t, oc, counts, rank, world, WANT_H32, device=dev,
                                     timings=timings if record else None)
            del ctx_out

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
    # PMC bytes per launch measured for THIS workload's pass-1 kernel (scripts/pmc_traffic.py)
    tf = os.path.join(ROOT, "profiles", "pass1_traffic.json" if args.workload == "config2"
                      else f"pass1_traffic_{args.workload}.json")
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get("workload", "config2") == args.workload:
                traffic = tj.get("hbm_bytes_per_launch")
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
        "data": f"synthetic (SURVEY.md §8(d) {args.workload} generator, seeded, generated in HBM)",
        "config": {"workload": f"{args.workload}: {B} "
                               f"{'dense' if args.workload == 'config3' else 'sparse'} "
                               f"traces/GPU x {M} B map, {args.mode} "
                               "classify+hash32+last-hash skip+has_new_bits, virgin carried",
                   "map_size": M, "batch_per_gpu": B, "global_batch": world * B,
                   "mode": args.mode, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": ("k_pass1w" if args.workload == "config3" else "k_pass1s"),
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


def _timed(fn, steps, warmup):
    import torch

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return el, sum(a.elapsed_time(b) for a, b in ev) / len(ev)


def main_merge(args):
    """BASELINE config 4: N client states (3 virgin maps of 64 KiB each) AND-folded into one
    (merger/merger.c:79-99), states resident in HBM; one step = one fold of all N.  Each state
    is all-0xff with random bits cleared (AND of 6 random bytes: P(clear) = 1/64)."""
    import torch

    from killerbeez_amd.triage import merge_and

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, sb = args.states, 3 * 65536
    states = torch.empty((n, sb), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed)
    for lo in range(0, n, 2000):
        hi = min(n, lo + 2000)
        clr = torch.randint(0, 256, (hi - lo, sb), dtype=torch.uint8, device=dev, generator=g)
        for _ in range(5):
            clr &= torch.randint(0, 256, (hi - lo, sb), dtype=torch.uint8, device=dev,
                                 generator=g)
        states[lo:hi] = ~clr
    out = torch.empty(sb, dtype=torch.uint8, device=dev)
    el, ms = _timed(lambda: merge_and(states, out=out), args.steps, args.warmup)
    torch.cuda.synchronize()
    # size-independent property: the fold equals the AND of the folds of the two halves
    halves = merge_and(states[: n // 2]) & merge_and(states[n // 2:])
    if not torch.equal(halves, out):
        raise SystemExit("merge self-check failed")
    bytes_ = n * sb
    res = {"metric": "merger states AND-folded/sec (3 x 64 KiB virgin maps per state)",
           "value": round(n * args.steps / el, 1), "unit": "states/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1e3 * el / args.steps, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic merger states (all-0xff, bits cleared w.p. 1/64), generated in HBM",
           "config": {"workload": f"config4: {n} states x {sb} B, one AND-fold per step",
                      "states": n, "state_bytes": sb, "parallelism": "shard1"},
           "roofline": {"bound": "hbm", "achieved": round(bytes_ / (ms * 1e-3) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(bytes_ / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None, "kernel": "k_and_groups + k_and_rows (one fold)",
                        "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": bytes_}}
    if not args.no_cpu:
        import oracle

        sample = states[:2000].cpu().numpy()
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            oracle.merge_many(sample)
            done += sample.shape[0]
        el_c = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": done / el_c, "unit": "states/s", "cores": 1,
                               "kind": "port",
                               "sample": f"2000 states of the workload, AND-folded repeatedly "
                                         f"({el_c:.1f} s), oracle kbzo_merge_many, 1 thread"}
    print(json.dumps(res), flush=True)


def main_stream(args):
    """BASELINE config 5 (1 GPU): config-2 traces in pageable host memory, triaged through
    kbz_triage_batch_host (pinned ring, double-buffered hipMemcpyAsync).  PCIe-bound; this is
    the PCIe-inclusive rate DESIGN.md quotes, never the headline value."""
    import torch

    from killerbeez_amd import synth
    from killerbeez_amd.triage import MODES, WANT_H32, TriageContext

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, M = min(args.batch, 16384), args.map_size
    t, oc = synth.sparse_torch(B, M, seed=args.seed, device=dev)
    host, hoc = t.cpu().numpy(), oc.cpu().numpy()
    del t, oc
    ctx = TriageContext(M, MODES[args.mode], B)
    for _ in range(args.warmup):
        ctx.triage_host(host, hoc, WANT_H32)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.triage_host(host, hoc, WANT_H32)
    el = time.perf_counter() - t0
    res = {"metric": "traces triaged/sec from host memory (64KB map, PCIe-inclusive)",
           "value": round(B * args.steps / el, 1), "unit": "traces/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1e3 * el / args.steps, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic config-2 traces in pageable host memory",
           "config": {"workload": f"stream: {B} sparse traces x {M} B per step via the pinned "
                                  "ring", "batch": B, "map_size": M, "mode": args.mode},
           "pcie_GBps": round(B * M * args.steps / el / 1e9, 2)}
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
