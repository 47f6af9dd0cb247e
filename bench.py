#!/usr/bin/env python3
"""Headline benchmark: traces triaged/s (64 KiB map, classify + novelty + hash32) on MI355X.

Workload (BASELINE.json configs[1]): per GPU, batches of 65,536
synthetic sparse traces x 64 KiB raw hit counters (seeded generator in killerbeez_amd.synth,
generated directly in HBM; every batch is a different sample of the same target program: they
share the hot edge set), triaged with DynamoRIO semantics (dynamorio_instrumentation.c:
1428-1468: classify_counts, hash32, last-hash skip, has_new_bits vs virgin_bits).  One step =
one full triage of one batch; the virgin map and last hash carry over from step to step.

`value` is measured on FRESH batches: every warmup and timed step triages a batch it has never
seen (pool = warmup + steps distinct batches, 4 GiB each), so the novelty scan and claim
resolution do real work.  Also reported ("variants"): the same steps on already-absorbed
batches (steady state: nothing new), fresh batches in which 90 % of execs repeat their
predecessor (the last-hash skip path), and the first batch on all-0xff virgin maps.

With --gpus N every rank triages its own 65,536-trace shard of an N x 65,536-trace global
batch with the exact sharded protocol of killerbeez_amd.dist (RCCL all-gathers) -- weak
scaling.  Without an outside launcher, `--gpus N` (N > 1) starts N ranks itself
(torch.distributed.run, 127.0.0.1) from a parent that never touches the GPU.

Prints ONE JSON line (rank 0).  Also reports the dominant kernel's (pass 1) achieved
algorithmic HBM bandwidth against the 8 TB/s peak (HIP events around each pass-1 launch), and
the reference CPU path timed on this host's cores on a bounded sample.

Other workloads: --workload config3 (16,384 dense x 1 MiB), merge (config 4: 100k merger
states AND-folded, sharded over the ranks), stream (config 5: traces from host memory through
the pinned ingest ring + the unique crash/hang table, PCIe-bound), plugin (per-exec latency of
the instrumentation plugin at batch sizes 1/16/256/4096).
"""
from __future__ import annotations

import argparse
import json

import numpy as np
import os
import shutil
import socket
import subprocess
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
    p.add_argument("--pool", type=int, default=0,
                   help="distinct batches (default warmup + steps, capped by free HBM)")
    p.add_argument("--repeat-frac", type=float, default=0.9)
    p.add_argument("--hash", action="store_true",
                   help="AFL modes: also compute hash32 (the reference AFL plugin never hashes, "
                        "afl_instrumentation.c:231-274; DynamoRIO mode always does)")
    p.add_argument("--no-variants", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-pmc", dest="pmc", action="store_false",
                   help="skip the live roofline.traffic measurement (two rocprofv3 --pmc passes "
                        "of a short child run, rank 0 with 1 GPU) and report the stored one")
    p.add_argument("--no-ktrace", dest="ktrace", action="store_false",
                   help="skip the rocprofv3 --kernel-trace child run behind roofline.rocprof "
                        "(rank 0 with 1 GPU)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--workload", default="config2",
                   choices=["config2", "config3", "merge", "stream", "plugin"])
    p.add_argument("--states", type=int, default=100000, help="merge workload: states (total)")
    p.add_argument("--no-selfcheck", dest="selfcheck", action="store_false",
                   help=argparse.SUPPRESS)  # PMC child runs: only the timed folds' kernels
    a = p.parse_args()
    if a.workload == "config3":
        if a.batch == 65536:
            a.batch = 16384
        if a.map_size == 65536:
            a.map_size = 1 << 20
    return a


# ---- launching ---------------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def maybe_launch(args):
    """--gpus N > 1 without an outside torch.distributed.run: start the N ranks as children
    (this process has not touched the GPU) and exit with their status."""
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        sys.exit(subprocess.call(cmd, env=env))


# Rehearsal of the multi-rank path on a one-GPU box (never for reported numbers): with
# KBZ_BENCH_REHEARSE=1 every rank uses cuda:0 and the collectives go through gloo (RCCL needs
# one GPU per rank).
REHEARSE = os.environ.get("KBZ_BENCH_REHEARSE") == "1"


def init_dist():
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local if world > 1 and not REHEARSE else 0)
    torch.cuda.set_device(dev)
    if world > 1:
        if REHEARSE:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    return world, rank, dev


def barrier_sync(world, dev):
    import torch
    import torch.distributed as dist

    torch.cuda.synchronize()
    if world > 1:
        if REHEARSE:
            dist.barrier()
        else:
            dist.barrier(device_ids=[dev.index])
    torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def finish(world):
    import torch.distributed as dist

    if dist.is_initialized():  # (world 1: the sharded-protocol variant's one-rank group)
        dist.destroy_process_group()


# ---- CPU baselines -----------------------------------------------------------------------------

def usable_cores():
    """Cores this process may run on: its affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) // float(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(traces_dev, outcome_dev, mode, seconds):
    """The reference's own per-exec novelty step (oracle/_ref: classify_counts + hash32 +
    has_new_bits in has_new_coverage's control flow for DynamoRIO; finish_fuzz_round's
    simplify + has_new_bits routing for AFL), one core, on a bounded sample of the same
    workload.  Falls back to the clean-room restatement if _ref is absent."""
    import ctypes as C

    import numpy as np

    import oracle

    m = traces_dev.shape[1]
    sample_n = min(traces_dev.shape[0], 8192 if m <= 65536 else 512)
    host = traces_dev[:sample_n].cpu().numpy()
    oc = outcome_dev[:sample_n].cpu().numpy().astype(np.int8)
    virgin = np.full(3 * m, 0xFF, np.uint8)
    scratch = np.empty(m, np.uint8)
    hnb = np.zeros(sample_n, np.uint8)
    last = C.c_uint32(0)
    sfx = {65536: "64k", 1 << 20: "1m"}.get(m)
    kind, fn = "port", None
    if sfx and oracle.have_ref() and mode in (0, 1):
        kind = "reference"
        args7 = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                 C.c_void_p]
        if mode == 1:
            f = getattr(oracle.ref(), f"ref_dr_triage_loop_{sfx}")
            f.argtypes = args7
            fn = lambda: f(host.ctypes.data, sample_n, m, virgin.ctypes.data, C.byref(last),
                           hnb.ctypes.data, scratch.ctypes.data)
        else:
            f = getattr(oracle.ref(), f"ref_afl_triage_loop_{sfx}")
            f.argtypes = args7
            fn = lambda: f(host.ctypes.data, sample_n, m, oc.ctypes.data, virgin.ctypes.data,
                           hnb.ctypes.data, scratch.ctypes.data)
    if fn is None:
        fn = lambda: oracle.triage_batch(mode, host, oc, threads=0)
    done, passes, t0 = 0, 0, time.perf_counter()
    while True:
        fn()
        done += sample_n
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    flags = ""
    if kind == "reference":
        try:
            rf = oracle.ref().ref_build_flags
            rf.restype = C.c_char_p
            flags = f", reference built with gcc {rf().decode()}"
        except AttributeError:
            flags = ", reference build flags unrecorded"
    return {"value": round(done / el, 1), "unit": "traces/s", "cores": 1, "kind": kind,
            "sample": f"{sample_n} traces x {m} B of the bench workload{flags}, {passes} sequential "
                      f"passes ({el:.1f} s), virgin carried, 1 thread"}


def cpu_baseline_all_cores(traces_dev, outcome_dev, mode, seconds):
    """Clean-room restatement, exact sharded decomposition over the usable host cores (port):
    two reads per trace (oracle/kbz_oracle.c kbzo_triage_batch_mt)."""
    import numpy as np

    import oracle

    threads = usable_cores()
    m = traces_dev.shape[1]
    sample_n = min(traces_dev.shape[0], 16384 if m <= 65536 else 1024)
    host = traces_dev[:sample_n].cpu().numpy()
    oc = outcome_dev[:sample_n].cpu().numpy().astype(np.int8)
    done, t0 = 0, time.perf_counter()
    while True:
        oracle.triage_batch(mode, host, oc, threads=threads)
        done += sample_n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    granted = oracle.cpu_cores_granted(threads)
    mem = {f"{t}_threads": round(oracle.host_read_gbps(t, host), 1) for t in (1, threads)}
    return {"value": round(done / el, 1), "unit": "traces/s", "cores": threads, "kind": "port",
            "cores_granted": round(granted, 2), "host_read_GBps": mem,
            "sample": f"{sample_n} traces, oracle/kbz_oracle.c kbzo_triage_batch_mt, "
                      f"{threads} threads (sched_getaffinity, cgroup quota); cores_granted = "
                      f"threads x t(1) / t(threads) of a register-only chain per thread"}


# ---- profiler children --------------------------------------------------------------------------
#
# Every profiler child (PMC passes, the kernel trace) is started by profile_first() BEFORE this
# process touches the GPU, and rocprofv3 (a `#!/usr/bin/env python3` script) is started as
# [sys.executable, rocprofv3] so no `env` hop execs anything.  The children themselves run with
# --no-pmc --no-ktrace: a profiled child never starts another profiler (round 4's PMC children
# did: their nested kernel-trace launches were the execs the GPU box refused).

def _rocprof():
    path = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return [sys.executable, path]


def _child_args():
    return [os.path.abspath(__file__), "--no-cpu", "--no-variants", "--no-pmc", "--no-ktrace"]


# ---- roofline traffic (PMC) --------------------------------------------------------------------

def _pmc_pass(counter, workload_args, outdir, timeout=150, kernel="k_pass1"):
    """One rocprofv3 --pmc pass over a short child run; per-dispatch values of `counter` for
    the kernels whose name contains `kernel` (default: pass 1), in launch order."""
    import csv
    import glob

    cmd = [*_rocprof(), "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "run",
           "--", sys.executable, *_child_args(), *workload_args]
    subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout,
                   check=True)
    vals = []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                vals.append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
    return [v for _, v in sorted(vals)]


def live_traffic(args, warmup=1, steps=4):
    """HBM bytes per pass-1 launch from PMC (MI355X_MICROARCH.md HBM section): FETCH_SIZE and
    WRITE_SIZE in separate passes (their TCC slots do not fit one pass), KiB per dispatch;
    FETCH_SIZE doubled (gfx950 tallies 16 B/lane streaming reads at half their bytes).  The
    median over the timed (fresh-batch) dispatches."""
    import tempfile

    wa = ["--workload", args.workload, "--mode", args.mode, "--batch", str(args.batch),
          "--map-size", str(args.map_size), "--warmup", str(warmup), "--steps", str(steps),
          "--seed", str(args.seed), *(["--hash"] if args.hash else [])]
    with tempfile.TemporaryDirectory() as d:
        fetch = _pmc_pass("FETCH_SIZE", wa, os.path.join(d, "f"))[warmup:]
        write = _pmc_pass("WRITE_SIZE", wa, os.path.join(d, "w"))[warmup:]
    if not fetch or not write:
        return None
    med = lambda v: sorted(v)[len(v) // 2]
    return {"bytes": 2.0 * med(fetch) * 1024 + med(write) * 1024,
            "source": f"live rocprofv3 --pmc, {len(fetch)} fresh-batch dispatches: "
                      f"FETCH_SIZE x2 = {2.0 * med(fetch) * 1024:.0f} B + WRITE_SIZE = "
                      f"{med(write) * 1024:.0f} B"}


def summarize_ktrace(csv_files, steps, kernel_prefix="k_pass1"):
    """Parse rocprofv3 kernel_trace.csv files of one run: the last `steps` dispatches whose name
    starts with `kernel_prefix` are its timed steps (runs without variants).  Returns
    (summary, per-step kernel lists, pass-1 durations in ms) or None."""
    import csv

    rows = []
    for f in csv_files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if "(anonymous namespace)::k_" not in name:
                continue
            k = name.split("(anonymous namespace)::")[1].split("(")[0].split("<")[0]
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), k))
    rows.sort()
    p1 = [i for i, x in enumerate(rows) if x[2].startswith(kernel_prefix)]
    if len(p1) < steps:
        return None
    first = p1[-steps]
    timed = [i for i in p1 if i >= first]
    durs = [(rows[i][1] - rows[i][0]) / 1e6 for i in timed]
    per_step = []
    for si, i in enumerate(timed):
        nxt = timed[si + 1] if si + 1 < len(timed) else len(rows)
        t0 = rows[i][0]
        per_step.append([{"kernel": rows[j][2], "start_us": round((rows[j][0] - t0) / 1e3, 2),
                          "dur_us": round((rows[j][1] - rows[j][0]) / 1e3, 2)}
                         for j in range(i, nxt)])
    span = [(rows[timed[si + 1]][0] - rows[i][0]) / 1e6 for si, i in enumerate(timed[:-1])]
    avg = sum(durs) / len(durs)
    out = {"avg_ms": round(avg, 4), "min_ms": round(min(durs), 4), "max_ms": round(max(durs), 4),
           "median_ms": round(sorted(durs)[len(durs) // 2], 4), "dispatches": len(durs),
           "median_step_span_ms": round(sorted(span)[len(span) // 2], 4) if span else None}
    return out, per_step, durs


def live_kernel_trace(args, warmup=3, steps=12):
    """The roofline's kernel time from the profiler: a rocprofv3 --kernel-trace child run of the
    same workload (no variants, no PMC); its timed steps' pass-1 dispatches are the last `steps`
    pass-1 dispatches of the trace.  Returns their average duration (and min / max), the child's
    own ms_per_step and HIP-event pass-1 time, and every kernel of those steps (start relative to
    the step's pass 1, duration), also written to $KBZ_BENCH_KTRACE_OUT (a JSON the evidence
    script commits under profiles/) -- so the line's `frac` can be recomputed from profiles/."""
    import glob
    import tempfile

    wa = ["--workload", args.workload, "--mode", args.mode, "--batch", str(args.batch),
          "--map-size", str(args.map_size), "--warmup", str(warmup), "--steps", str(steps),
          "--seed", str(args.seed), *(["--hash"] if args.hash else [])]
    with tempfile.TemporaryDirectory() as d:
        cmd = [*_rocprof(), "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run",
               "--", sys.executable, *_child_args(), *wa]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True)
        child = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        got = summarize_ktrace(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"),
                                         recursive=True), steps)
    if got is None:
        return None
    out, per_step, durs = got
    out.update({"child_ms_per_step": child.get("ms_per_step"),
                "child_hip_event_avg_ms": child.get("roofline", {}).get("avg_launch_ms"),
                "what": f"rocprofv3 --kernel-trace of a child run of this workload ({warmup} "
                        f"warmup + {steps} timed fresh batches), started before this process "
                        f"touched the GPU; the last {steps} pass-1 dispatches = its timed steps; "
                        "step span = pass-1 start to the next pass-1 start"})
    dest = os.environ.get("KBZ_BENCH_KTRACE_OUT")
    if dest:
        os.makedirs(os.path.dirname(os.path.abspath(dest)), exist_ok=True)
        json.dump(dict(out, workload=args.workload, mode=args.mode, batch=args.batch,
                       map_size=args.map_size, pass1_durations_ms=[round(x, 5) for x in durs],
                       steps=per_step), open(dest, "w"), indent=1)
        out["trace_file"] = dest
    return out


# A/B only: KBZ_BENCH_P1_TIMING=0 times the steps without the pass-1 events (roofline invalid)
P1_TIMING = os.environ.get("KBZ_BENCH_P1_TIMING", "1") != "0"
# A/B only: KBZ_BENCH_P1_EVERY=k times one pass-1 launch in k (events on a dispatch leave ~5 us
# of idle GPU behind it in a kernel trace, profiles/r05_evgap; sampling 1 in 4 did not change
# ms_per_step beyond the ±2 % between processes, profiles/r05_every): default every launch
P1_EVERY = max(1, int(os.environ.get("KBZ_BENCH_P1_EVERY", "1")))
VALU_ISSUE_CYCLES = 4  # one wave64 integer VALU instruction per SIMD per 4 cycles (tools/xprobe,
                       # SQ_ACTIVE_INST_VALU = SQ_INSTS_VALU quad-cycles: profiles/r03_v8)
SIMDS = 256 * 4
CLOCK_PEAK_GHZ = 2.4


def live_valu(args, warmup=1, steps=2):
    """Config 3's pass 1 is VALU-issue-bound, not HBM-bound: the VALU instructions of one launch
    (SQ_INSTS_VALU, all waves) and the time they take if all 1,024 SIMDs issued one every 4
    cycles at the peak clock -- the instruction-count floor the kernel is measured against."""
    import tempfile

    wa = ["--workload", args.workload, "--mode", args.mode, "--batch", str(args.batch),
          "--map-size", str(args.map_size), "--warmup", str(warmup), "--steps", str(steps),
          "--seed", str(args.seed), *(["--hash"] if args.hash else [])]
    with tempfile.TemporaryDirectory() as d:
        v = _pmc_pass("SQ_INSTS_VALU", wa, os.path.join(d, "v"))[warmup:]
    if not v:
        return None
    inst = sorted(v)[len(v) // 2]
    floor_ms = inst * VALU_ISSUE_CYCLES / SIMDS / (CLOCK_PEAK_GHZ * 1e6)
    return {"instructions_per_launch": inst, "floor_ms": round(floor_ms, 4),
            "what": f"SQ_INSTS_VALU (live rocprofv3 --pmc, median of {len(v)} fresh-batch "
                    f"dispatches) x {VALU_ISSUE_CYCLES} cycles / {SIMDS} SIMDs at "
                    f"{CLOCK_PEAK_GHZ} GHz"}


def merge_traffic(args, warmup=1, steps=3):
    """HBM bytes of one local AND-fold of the merge leg (k_and_groups tree + k_and_rows), from
    PMC like live_traffic: the fold kernels' per-dispatch FETCH_SIZE x2 + WRITE_SIZE summed over
    the timed steps, divided by the steps (the first `warmup` steps' kernels are skipped)."""
    import tempfile

    wa = ["--workload", "merge", "--states", str(args.states), "--warmup", str(warmup),
          "--steps", str(steps), "--seed", str(args.seed), "--no-selfcheck"]
    with tempfile.TemporaryDirectory() as d:
        fetch = _pmc_pass("FETCH_SIZE", wa, os.path.join(d, "f"), kernel="k_and_")
        write = _pmc_pass("WRITE_SIZE", wa, os.path.join(d, "w"), kernel="k_and_")
    per = len(fetch) // (warmup + steps)  # every step launches the same fold kernels
    if not fetch or not write or per == 0:
        return None
    tot = 2.0 * sum(fetch[per * warmup:per * (warmup + steps)]) * 1024 + \
        sum(write[per * warmup:per * (warmup + steps)]) * 1024
    return {"bytes": tot / steps,
            "source": f"live rocprofv3 --pmc: FETCH_SIZE x2 + WRITE_SIZE of the {per} fold "
                      f"kernels of each of {steps} steps"}


def stored_traffic(workload):
    """The last committed PMC measurement for this workload (profiles/pass1_traffic*.json)."""
    tf = os.path.join(ROOT, "profiles", "pass1_traffic.json" if workload == "config2"
                      else f"pass1_traffic_{workload}.json")
    try:
        tj = json.load(open(tf))
    except (OSError, ValueError):
        return None
    if tj.get("workload", "config2") != workload:
        return None
    return {"bytes": tj.get("hbm_bytes_per_launch"),
            "source": f"stored PMC measurement {os.path.relpath(tf, ROOT)} "
                      f"({tj.get('tag', 'earlier run')}), not this run"}


# ---- triage workloads (config 2 / config 3) ----------------------------------------------------

def crash_variant(args, pool, barrier_sync, dev, steps=5):
    """SURVEY.md §8(d) 'simplify-mode (crash) variant': the same traces triaged in AFL mode with
    every exec a crash (finish_fuzz_round, afl_instrumentation.c:260-265: simplify_trace, then
    has_new_bits against virgin_crash), on a context of its own."""
    import torch

    from killerbeez_amd.triage import MODES, WANT_H32, TriageContext

    B, M = args.batch, args.map_size
    want = WANT_H32 if args.hash else 0  # the reference AFL plugin never hashes
    crash = torch.full((B,), 2, dtype=torch.int8, device=dev)  # KBZ_FUZZ_CRASH
    with TriageContext(M, MODES["afl"], B) as c2:
        out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev)}
        if want:
            out["h32"] = torch.empty(B, dtype=torch.int32, device=dev)
        c2.triage(pool[0][0], crash, want, out=out)  # warmup
        barrier_sync(1, dev)
        c2.sync()
        c2.time_pass1(True)
        t0 = time.perf_counter()
        for i in range(steps):
            c2.triage(pool[(i + 1) % len(pool)][0], crash, want, out=out)
        barrier_sync(1, dev)
        el = time.perf_counter() - t0
        ms, launches = c2.time_pass1(False)
        c2.sync()
    return {"value": round(B * steps / el, 1), "ms_per_step": round(1e3 * el / steps, 4),
            "pass1_ms": round(ms / max(1, launches), 4),
            "what": f"{steps} batches of the pool in AFL mode, every exec a crash (simplify + "
                    f"virgin_crash), own context, {'with' if want else 'no'} hash32"}


def novelty_heavy(args, mode, want, batches, dev, steps=8):
    """Campaign starts, new targets, freshly merged states: every step triages a never-seen batch
    against all-0xff virgin maps, on a context of its own that already ran one such batch
    (first-launch costs excluded).  Timed like the headline: `steps` back-to-back steps between
    two synchronisations, each step = a stream-ordered reset of the virgin maps to 0xff
    (kbz_reset_virgin, 192 KiB memset, included in the time) + the triage, HIP events on pass 1.
    The stage breakdown comes from one extra untimed step with stage events on (they add gaps)."""
    import torch

    from killerbeez_amd.triage import TriageContext

    B, M = args.batch, args.map_size
    with TriageContext(M, mode, B) as c:
        out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev)}
        if want:
            out["h32"] = torch.empty(B, dtype=torch.int32, device=dev)
        c.reset_virgin()
        c.triage(*batches[0], want, out=out)  # warm: first launches, allocations
        c.sync()
        c.reset_virgin()
        c.time_stages(True)
        c.triage(*batches[1 % len(batches)], want, out=out)
        stages, _ = c.time_stages(False)
        c.sync()
        claims = c.stats()["claims"]
        torch.cuda.synchronize()
        c.time_pass1(True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(steps):
            t, oc = batches[(i + 2) % len(batches)]
            c.reset_virgin()
            c.triage(t, oc, want, out=out)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / steps
        p1ms, nl = c.time_pass1(False)
        p1 = p1ms / max(1, nl)
        c.sync()
        # continuity with round 4's figure: steps one at a time (synchronised between steps, the
        # reset outside the events; round 4 also had stage events on inside them)
        iso = []
        for i in range(3):
            t, oc = batches[(i + 2 + steps) % len(batches)]
            c.reset_virgin()
            torch.cuda.synchronize()
            a.record()
            c.triage(t, oc, want, out=out)
            b.record()
            b.synchronize()
            iso.append(a.elapsed_time(b))
        c.sync()
    return {"ms_per_step": round(ms, 4), "pass1_ms": round(p1, 4),
            "isolated_step_ms": round(sum(iso) / len(iso), 4),
            "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            "claims_per_batch": int(claims),
            "what": f"{steps} never-seen batches back to back, each on all-0xff virgin maps "
                    "(stream-ordered reset inside the timed steps), own warmed-up context; "
                    "stage_ms from one extra untimed step with stage events"}


def sharded_world1(args, ctx, batches, counts, want, dev, snap, fused_ms):
    """The N > 1 step at N = 1: the headline's fresh batches through dist.triage_sharded with
    force_collective on a one-rank RCCL communicator (both all-gathers run), so the protocol's
    cost over the fused one-shard step is measured on a one-GPU box; phase times from HIP
    events around each phase.  Each timed pass starts from `snap` (the virgin maps and last hash
    the headline's timed steps started from), so it does the headline's work: the same batches,
    never seen, in the same order."""
    import torch
    import torch.distributed as dist

    from killerbeez_amd.dist import timing_summary, triage_sharded

    try:
        if not dist.is_initialized():
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}",
                                    rank=0, world_size=1, device_id=dev)
        log = []
        el_box = {}

        def sharded_step(t, oc):
            triage_sharded(ctx, t, oc, counts[:1], 0, 1, want, device=dev, timings=log,
                           force_collective=True)

        def restore():
            torch.cuda.synchronize()
            ctx.set_virgin(snap[0])
            ctx.last_hash = snap[1]
            torch.cuda.synchronize()

        # warm the communicator and the staged kernels, then the timed steps (phase events on)
        for t, oc in batches[:2]:
            sharded_step(t, oc)
        torch.cuda.synchronize()
        log.clear()
        restore()
        t0 = time.perf_counter()
        for i in range(args.steps):
            sharded_step(*batches[i % len(batches)])
        torch.cuda.synchronize()
        el_box["s"] = time.perf_counter() - t0
        phases = timing_summary(log)
        # the same steps without phase events (the events add their own gaps)
        restore()
        t0 = time.perf_counter()
        for i in range(args.steps):
            triage_sharded(ctx, *batches[i % len(batches)], counts[:1], 0, 1, want, device=dev,
                           force_collective=True)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / args.steps
        return {"ms_per_step": round(ms, 4), "fused_ms_per_step": round(fused_ms, 4),
                "extra_us_per_step": round(1e3 * (ms - fused_ms), 1),
                "ms_per_step_with_phase_events": round(1e3 * el_box["s"] / args.steps, 4),
                "phase_ms": {k: round(v, 4) for k, v in phases.items()},
                "backend": dist.get_backend(),
                "what": "the headline's fresh batches through triage_sharded(force_collective="
                        "True) on a one-rank RCCL group (the N>1 step's kernels and both "
                        "all-gathers), each pass from the virgin maps and last hash the headline "
                        "started from; fused_ms_per_step = the headline's step"}
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"[:300]}


def main_triage(args, pre):
    import torch

    from killerbeez_amd import synth
    from killerbeez_amd.dist import timing_summary, triage_sharded
    from killerbeez_amd.triage import MODES, WANT_H32, TriageContext

    world, rank, dev = init_dist()
    mode = MODES[args.mode]
    B, M = args.batch, args.map_size
    dense = args.workload == "config3"
    gen = synth.dense_torch if dense else synth.sparse_torch
    want_pool = args.pool or (args.warmup + args.steps)
    free, _ = torch.cuda.mem_get_info(dev)
    cap = max(2, int(0.6 * free) // (B * M))  # room left for the context and the variants
    npool = max(2, min(want_pool, cap))
    pool = [gen(B, M, seed=args.seed + 7919 * p + 104729 * rank, device=dev, hot_seed=args.seed)
            for p in range(npool)]
    ctx = TriageContext(M, mode, B)
    # DynamoRIO always hashes (last-hash skip); the AFL plugin never does unless asked
    want = WANT_H32 if (mode == MODES["dynamorio"] or args.hash) else 0
    out = {"hnb": torch.empty(B, dtype=torch.uint8, device=dev)}
    if want:
        out["h32"] = torch.empty(B, dtype=torch.int32, device=dev)
    counts = [B] * world
    timed_launches = []  # pass-1 launches timed by each timed() call
    phase_log = None  # list: per-batch phase timings of the sharded protocol (world > 1)

    def step(t, oc):
        if world == 1:  # one shard: kbz_triage_batch_device (pass 1 [+ k_skip], k_tail, k_fin)
            ctx.triage(t, oc, want, out=out)
        else:
            triage_sharded(ctx, t, oc, counts, rank, world, want, device=dev, timings=phase_log)

    def timed(batches, k, events=False):
        """k steps over batches[i % len], bracketed by barrier + synchronize; max over ranks.
        Returns (seconds, pass-1 ms per launch[, device ms of the k steps]).  Stage timing (two
        events per stage) stays off here: it adds ~50 us per step; the warmup steps time stages."""
        barrier_sync(world, dev)
        ctx.sync()
        ctx.time_pass1_every(P1_EVERY)
        ctx.time_pass1(P1_TIMING)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0 = time.perf_counter()
        ev[0].record()
        for i in range(k):
            step(*batches[i % len(batches)])
        ev[1].record()
        barrier_sync(world, dev)
        el = time.perf_counter() - t0
        ms, launches = ctx.time_pass1(False)
        ctx.time_pass1_every(1)
        ctx.sync()
        timed_launches.append(launches)
        r = (max_over_ranks(el, world, dev), ms / launches if launches else float("nan"))
        return r + (ev[0].elapsed_time(ev[1]),) if events else r

    # warmup on fresh batches (the first one on all-0xff virgin maps, timed by itself); the
    # other warmup batches are fresh too and time the stages after pass 1
    _, _, cold_ms = timed(pool[:1], 1, events=True)
    ctx.time_stages(True)
    for i in range(1, args.warmup):
        step(*pool[i % npool])
    st, nb = ctx.time_stages(False)
    stage_ms = {k2: round(v / max(1, nb), 4) for k2, v in st.items()}
    fresh = pool[args.warmup:] if npool > args.warmup else pool
    phase_log = [] if world > 1 else None
    # the state the timed fresh steps start from (the sharded variant replays them from it)
    snap = None
    if world == 1 and not args.no_variants and not dense:
        torch.cuda.synchronize()
        snap = (ctx.get_virgin(), ctx.last_hash)
    elapsed, pass1_ms = timed(fresh, args.steps)
    pass1_timed = timed_launches[-1]
    phases = timing_summary(phase_log) if phase_log else {}
    phase_log = None
    n_fresh = min(args.steps, len(fresh))
    fresh_stats = ctx.stats()  # work of the last timed batch (claim items resolved, ...)
    value = world * B * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    achieved = B * M / (pass1_ms * 1e-3) / 1e9  # GB/s, algorithmic bytes of one launch
    variants = {"cold_first_batch_ms": round(cold_ms, 4),
                "last_fresh_batch_work": fresh_stats,
                "stage_ms_per_step": stage_ms,
                "stage_ms_note": "fresh warmup batches 2..W, stage events on (off in the timed steps)"}
    if snap is not None:  # before the variants below mutate or re-triage the batches
        variants["sharded_protocol_world1"] = sharded_world1(
            args, ctx, fresh[:args.steps], counts, want, dev, snap, ms_per_step)
    if not args.no_variants:
        seen = pool[-2:]
        el2, p2 = timed(seen, args.steps)
        variants["steady_state_seen_batches"] = {
            "value": round(world * B * args.steps / el2, 1),
            "ms_per_step": round(1e3 * el2 / args.steps, 4), "pass1_ms": round(p2, 4),
            "what": "the same steps re-triaging 2 already absorbed batches (nothing new)"}
        if mode == MODES["dynamorio"]:
            reps = 0
            rb = fresh[:max(1, min(len(fresh), args.steps))]
            for i, (t, oc) in enumerate(rb):
                reps += synth.with_repeats_torch(t, oc, args.repeat_frac,
                                                 seed=args.seed + 31 * i + rank)
            el3, p3 = timed(rb, args.steps)
            st = ctx.stats()
            variants[f"repeats{int(round(100 * args.repeat_frac))}"] = {
                "value": round(world * B * args.steps / el3, 1),
                "ms_per_step": round(1e3 * el3 / args.steps, 4), "pass1_ms": round(p3, 4),
                "rest_of_step_ms": round(1e3 * el3 / args.steps - p3, 4),
                "repeated_execs": reps, "last_batch_fixed_chunks": st["fixed_chunks"],
                "what": f"{len(rb)} of the fresh batches with {args.repeat_frac:.0%} of execs "
                        "repeating their predecessor (last-hash skips), virgin carried"}
        if world == 1:
            variants["afl_all_crash_simplify"] = crash_variant(args, pool, barrier_sync, dev)
            variants["novelty_heavy"] = novelty_heavy(args, mode, want, fresh, dev)
    del pool, fresh
    traffic = pre["traffic"]
    if traffic is None:
        traffic = stored_traffic(args.workload) or {"bytes": None, "source": "none"}
    ktrace, valu = pre["ktrace"], pre["valu"]
    wide = B < 512 * 64
    if mode == MODES["dynamorio"]:
        kname = "k_pass1d" if wide else "k_pass1s"
    elif want:
        kname = "k_pass1w" if wide else "k_pass1s"
    else:
        kname = "k_pass1n (wide)" if wide else "k_pass1n"
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
        "data": f"synthetic (SURVEY.md §8(d) {args.workload} generator, seeded, generated in HBM; "
                f"{n_fresh} distinct never-seen batches in the timed steps)",
        "config": {"workload": f"{args.workload}: {B} {'dense' if dense else 'sparse'} "
                               f"traces/GPU x {M} B map, {args.mode} "
                               + ("classify+hash32+last-hash skip+has_new_bits"
                                  if mode == MODES["dynamorio"] else
                                  ("classify" if args.mode == "afl_classify" else "raw") +
                                  "/simplify+has_new_bits vs 3 virgin maps" +
                                  ("+hash32" if want else " (no hash, as the AFL plugin)")) +
                               ", virgin carried, fresh batches",
                   "map_size": M, "batch_per_gpu": B, "global_batch": world * B,
                   "mode": args.mode, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic["bytes"], "traffic_source": traffic["source"],
                     "kernel": kname,
                     "avg_launch_ms": round(pass1_ms, 4),
                     "timed_launches": pass1_timed,
                     "timed_launches_note": f"HIP events on one pass-1 launch in {P1_EVERY} of "
                                            "the timed steps",
                     "algorithmic_bytes_per_launch": B * M},
        "pass1_share_of_step": round(pass1_ms / ms_per_step, 4),
        "variants": variants,
    }
    if ktrace:
        if ktrace.get("avg_ms"):
            res["roofline"]["rocprof_avg_ms"] = ktrace["avg_ms"]
            res["roofline"]["rocprof_frac"] = round(B * M / (ktrace["avg_ms"] * 1e-3) / 1e9
                                                    / HBM_PEAK_GBS, 4)
        res["roofline"]["rocprof"] = ktrace
    if valu and valu.get("instructions_per_launch"):
        valu["frac"] = round(valu["floor_ms"] / pass1_ms, 4)
        valu["bound"] = "valu"
        res["roofline"]["valu_issue"] = valu
    if world > 1:
        # attribution of a sub-linear curve: every rank's pass-1 time and the time its steps
        # spent in the all-gathers (HIP events around each phase of the timed steps)
        import torch.distributed as dist

        mine = torch.tensor([pass1_ms, phases.get("collective", 0.0), phases.get("pass1", 0.0)],
                            dtype=torch.float64, device=dev)
        allv = torch.empty(world * 3, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allv, mine)
        allv = allv.view(world, 3).cpu().tolist()
        res["per_rank_pass1_ms"] = [round(v[0], 4) for v in allv]
        res["collective_ms"] = {"max_over_ranks": round(max(v[1] for v in allv), 4),
                                "per_rank": [round(v[1], 4) for v in allv],
                                "what": "mean per step of the rank's all-gathers (DynamoRIO "
                                        "last row + hash, aggregates), HIP events"}
        res["phase_ms_rank0"] = {k: round(v, 4) for k, v in phases.items()}
        res["rccl_world"] = {"world_size": world, "backend": dist.get_backend(),
                             "rehearsal_one_gpu": REHEARSE}
    if rank == 0 and world == 1 and not args.no_cpu:
        t0, oc0 = gen(min(B, 16384), M, seed=args.seed + 1, device=dev, hot_seed=args.seed)
        res["cpu_baseline"] = cpu_baseline(t0, oc0, mode, args.cpu_seconds)
        res["cpu_baseline_all_cores"] = cpu_baseline_all_cores(t0, oc0, mode,
                                                               max(2.0, args.cpu_seconds / 3))
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    finish(world)


# ---- config 4: merger --------------------------------------------------------------------------

def main_merge(args, pre):
    """BASELINE config 4: N client states (3 virgin maps of 64 KiB each) AND-folded into one
    (merger/merger.c:79-99), states resident in HBM, split evenly over the ranks (strong
    scaling: the N states are the job); one step = one fold of all N (local fold, all-gather of
    the partial folds, local AND: killerbeez_amd.dist.merge_sharded).  Each state is all-0xff
    with random bits cleared (AND of 6 random bytes: P(clear) = 1/64)."""
    import torch

    from killerbeez_amd.dist import merge_sharded, split_counts
    from killerbeez_amd.triage import merge_and

    world, rank, dev = init_dist()
    n_all, sb = args.states, 3 * 65536
    counts = split_counts(n_all, world)
    n = counts[rank]
    states = torch.empty((n, sb), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + rank)
    for a in range(0, n, 2000):
        b = min(n, a + 2000)
        clr = torch.randint(0, 256, (b - a, sb), dtype=torch.uint8, device=dev, generator=g)
        for _ in range(5):
            clr &= torch.randint(0, 256, (b - a, sb), dtype=torch.uint8, device=dev, generator=g)
        states[a:b] = ~clr
    out = torch.empty(sb, dtype=torch.uint8, device=dev)
    fold_ev = []

    def step(record=False):
        if record:
            e = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
            e[0].record()
        local = merge_and(states)
        if record:
            e[1].record()
            fold_ev.append(e)
        merge_sharded(local.view(1, sb), world, out=out)

    for _ in range(args.warmup):
        step()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    ms = sum(a.elapsed_time(b) for a, b in fold_ev) / len(fold_ev)
    if world == 1 and args.selfcheck:  # size-independent: the fold = AND of the halves' folds
        halves = merge_and(states[: n // 2]) & merge_and(states[n // 2:])
        if not torch.equal(halves, out):
            raise SystemExit("merge self-check failed")
    bytes_ = n * sb
    traffic = {"bytes": None, "source": "not measured (--no-pmc or N > 1)"}
    res = {"metric": "merger states AND-folded/sec (3 x 64 KiB virgin maps per state)",
           "value": round(n_all * args.steps / el, 1), "unit": "states/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1e3 * el / args.steps, 4), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic merger states (all-0xff, bits cleared w.p. 1/64), generated in HBM",
           "config": {"workload": f"config4: {n_all} states x {sb} B over {world} GPU(s), one "
                                  "AND-fold per step (local fold + all-gather + local AND)",
                      "states": n_all, "state_bytes": sb, "parallelism": f"shard{world}"},
           "roofline": {"bound": "hbm", "achieved": round(bytes_ / (ms * 1e-3) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(bytes_ / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": traffic["bytes"], "traffic_source": traffic["source"],
                        "kernel": "k_and_groups + k_and_rows (one local fold)",
                        "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": bytes_}}
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = merge_cpu_baseline(states, args.cpu_seconds)
    if pre["traffic"] is not None:
        res["roofline"]["traffic"] = pre["traffic"]["bytes"]
        res["roofline"]["traffic_source"] = pre["traffic"]["source"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    finish(world)


def merge_cpu_baseline(states, seconds):
    """The reference's own merge_bitmaps (afl_instrumentation.c:116-121) in the merger's fold
    order (merger/merger.c:79-99 -> afl_merge :123-140; oracle/_ref ref_afl_merge_loop), one
    core, on 2,000 states of the workload (JSON decode excluded: its encoding is external)."""
    import ctypes as C

    import numpy as np

    import oracle

    sample = states[:2000].cpu().numpy()
    acc = np.full(sample.shape[1], 0xFF, np.uint8)
    if oracle.have_ref():
        f = oracle.ref().ref_afl_merge_loop_64k
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        fn, kind = (lambda: f(acc.ctypes.data, sample.ctypes.data, sample.shape[0])), "reference"
    else:
        fn, kind = (lambda: oracle.merge_many(sample)), "port"
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        done += sample.shape[0]
    el = time.perf_counter() - t0
    return {"value": round(done / el, 1), "unit": "states/s", "cores": 1, "kind": kind,
            "sample": f"{sample.shape[0]} states of the workload AND-folded repeatedly "
                      f"({el:.1f} s), merge_bitmaps in merger.c's fold order, 1 thread"}


# ---- config 5: streaming ingest + unique crash/hang table --------------------------------------

def main_stream(args, pre=None):
    """BASELINE config 5: config-2 traces in pageable host memory, produced into the pinned
    ingest ring (kbz_ring_acquire/submit: double-buffered hipMemcpyAsync, triage with XXH64)
    and the crash/hang traces' keys {XXH64, outcome class} inserted into the unique crash/hang
    table, replicated on every rank (killerbeez_amd.dist.dedup_sharded: all-gather of the keys
    in global trace order).  PCIe-bound; `value` = traces/s over all ranks, host to results."""
    import numpy as np
    import torch

    from killerbeez_amd import synth
    from killerbeez_amd.dist import dedup_sharded
    from killerbeez_amd.triage import MODES, WANT_H32, WANT_X64, TriageContext, UniqueSet

    world, rank, dev = init_dist()
    M = args.map_size
    t, oc = synth.sparse_torch(16384, M, seed=args.seed + 104729 * rank, device=dev,
                               hot_seed=args.seed)
    host, hoc = t.cpu().numpy(), oc.cpu().numpy().astype(np.int8)
    del t, oc
    ctx = TriageContext(M, MODES[args.mode], min(args.batch, 4096))
    table = UniqueSet(1 << 20)
    rows, _ = ctx.ring_acquire()
    slot = rows.shape[0]
    ctx.ring_submit(0, False)
    ctx.ring_flush()
    pending = []  # (hnb, h32, x64, outcome) of submitted slots, filled on re-acquire / flush
    n_new = 0

    def dedup(item):
        nonlocal n_new
        _, _, x64, o = item
        keys = torch.from_numpy(np.stack([x64.view(np.int64), o.astype(np.int64)], 1)).to(dev)
        mask = torch.from_numpy(o != 0).to(dev)
        # every rank's slot is `slot` rows: a fixed cap, no host sync
        n_new = n_new + dedup_sharded(table, keys, mask, rank, world, cap=slot).sum()

    def step(i):
        r, o = ctx.ring_acquire()  # waits for this slot's previous batch: its results are in
        if len(pending) >= 2:
            dedup(pending.pop(0))
        lo = (i * slot) % (host.shape[0] - slot + 1)
        torch.from_numpy(r[:slot]).copy_(torch.from_numpy(host[lo:lo + slot]))  # threaded
        o[:slot] = hoc[lo:lo + slot]
        res = (np.empty(slot, np.uint8), np.empty(slot, np.uint32), np.empty(slot, np.uint64),
               hoc[lo:lo + slot].copy())
        ctx.ring_submit(slot, True, res[0], res[1], res[2], WANT_H32 | WANT_X64)
        pending.append(res)

    def drain():
        ctx.ring_flush()
        while pending:
            dedup(pending.pop(0))

    for i in range(args.warmup):
        step(i)
    drain()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    drain()
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    traces = world * slot * args.steps
    pcie = pcie_h2d_peak(dev)
    gbps = slot * M * args.steps / el / 1e9
    ins = table_insert_rate(dev)
    res = {"metric": "traces triaged/sec from host memory (64KB map, PCIe-inclusive) + unique "
                     "crash/hang table",
           "value": round(traces / el, 1), "unit": "traces/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1e3 * el / args.steps, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic config-2 traces in pageable host memory",
           "config": {"workload": f"stream: {slot} sparse traces x {M} B per step and GPU via the "
                                  "pinned ring, XXH64 keys of crash/hang traces into the "
                                  "replicated unique table", "slot": slot, "map_size": M,
                      "mode": args.mode, "parallelism": f"shard{world}"},
           "pcie_GBps_per_gpu": round(gbps, 2),
           "pcie_h2d_peak_GBps": pcie,
           "pcie_frac": round(gbps / pcie["value"], 4),
           "xxh64_table_insert": ins,
           "unique_crash_hang_keys": table.size(), "new_keys_reported": int(n_new)}
    ctx.close()
    if world == 1:
        res["multi_device_host_batch"] = multi_device_host_batch(args, host, hoc, pcie)
    if rank == 0:
        print(json.dumps(res), flush=True)
    finish(world)


def multi_device_host_batch(args, host, hoc, pcie, reps=3):
    """The one-process sharded path from C (kbz_triage_batch_devices): a pageable host batch
    split over workers, each staged on its own host thread through pinned slots, then the
    sharded protocol over the workers' devices.  Workers: every visible GPU, or 1 and 2 workers
    sharing cuda:0 on a one-GPU box (one PCIe link).  Reported against the pinned H2D peak of
    the same run (per link)."""
    import torch

    from killerbeez_amd.triage import MODES, WANT_H32, MultiTriageContext

    ngpu = torch.cuda.device_count()
    layouts = [list(range(ngpu))] if ngpu > 1 else [[0], [0, 0]]
    out = {}
    M, n = args.map_size, host.shape[0]
    for devs in layouts:
        try:
            with MultiTriageContext(M, MODES[args.mode], -(-n // len(devs)), devices=devs) as mc:
                mc.triage_host(host, hoc, WANT_H32)  # warm: staging slots, contexts
                best = float("inf")
                for _ in range(reps):
                    t0 = time.perf_counter()
                    mc.triage_host(host, hoc, WANT_H32)
                    best = min(best, time.perf_counter() - t0)
                gbps = n * M / best / 1e9
                links = len(set(devs))
                out[f"workers{len(devs)}_gpus{links}"] = {
                    "traces_per_s": round(n / best, 1), "GBps": round(gbps, 2),
                    "frac_of_pinned_h2d_peak": round(gbps / (links * pcie["value"]), 4),
                    "peer_pairs": mc.peer_pairs()}
        except Exception as e:  # noqa: BLE001
            out[f"workers{len(devs)}"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    out["what"] = (f"{n} traces x {M} B from pageable host memory per call (best of {reps}), "
                   "host to results, virgin carried; peak = pinned H2D per GPU link")
    return out


def pcie_h2d_peak(dev, mib=256, reps=8):
    """SURVEY.md §8(d) row 5's ceiling, measured in the same run: a pinned-host -> HBM
    hipMemcpyAsync of `mib` MiB, best of `reps` (HIP events on the copy's stream)."""
    import torch

    n = mib << 20
    src = torch.empty(n, dtype=torch.uint8).pin_memory()
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dst.copy_(src, non_blocking=True)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return {"value": round(n / (best * 1e-3) / 1e9, 2), "unit": "GB/s",
            "what": f"pinned {mib} MiB hipMemcpyAsync H2D, best of {reps}"}


def table_insert_rate(dev, n=1 << 20, batches=8):
    """Inserts/s of the unique crash/hang table (kbz_set_insert_device, ordered insert-if-absent)
    for batches of n random keys into a set sized for all of them (device-resident keys)."""
    import torch

    from killerbeez_amd.triage import UniqueSet

    g = torch.Generator(device=dev)
    g.manual_seed(5)
    keys = [torch.randint(-2**62, 2**62, (n, 2), dtype=torch.int64, device=dev, generator=g)
            for _ in range(batches)]
    table = UniqueSet(n * batches)
    table.insert(keys[0][:1024])  # warm
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in keys:
        table.insert(k)
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b)
    return {"value": round(n * batches / (ms * 1e-3), 1), "unit": "keys/s",
            "what": f"{batches} ordered batches of {n} random 16-B keys into one table"}


# ---- plugin per-exec latency -------------------------------------------------------------------

def plugin_loop_c(name, t, oc, M, pool_rows=2048):
    """tools/plugin_loop (built by build()) in a child process, one run per batch size."""
    import subprocess
    import tempfile

    from killerbeez_amd import build

    if not os.path.exists(build.PLUGIN_LOOP):
        raise SystemExit(f"{build.PLUGIN_LOOP} is missing: run build() first")
    dr = name == "dynamorio"
    out = {"by_batch": {}}
    with tempfile.TemporaryDirectory() as d:
        pf, of = os.path.join(d, "pool.bin"), os.path.join(d, "oc.bin")
        t[:pool_rows].tofile(pf)
        oc[:pool_rows].astype(np.int8).tofile(of)
        for bs, execs in ((1, 512 if dr else 4096), (16, 4096), (256, 8192), (4096, 16384)):
            r = subprocess.run([build.PLUGIN_LOOP, name, pf, of, str(M), str(pool_rows),
                                str(execs), str(bs)], capture_output=True, text=True, timeout=300)
            if r.returncode:
                raise SystemExit(f"plugin_loop failed: {r.stderr[-500:]}")
            out["by_batch"].update(json.loads(r.stdout)["by_batch"])
    return out


def main_plugin(args, pre=None):
    """Per-exec latency of the instrumentation plugin (libkbz_plugin.so, include/kbz_plugin.h)
    driven like fuzzer/main.c:370-418: every exec's raw trace is recorded, its novelty queried.
    Batch 1 = the unmodified per-exec loop (is_new_path after each exec flushes a batch of one);
    batch B = record B execs, then query their results (one GPU batch).  Reported next to the
    reference's own per-exec step on one core (oracle/_ref)."""
    import ctypes as C

    import torch

    from killerbeez_amd import build, synth

    M = args.map_size
    name = "dynamorio" if args.mode == "dynamorio" else "afl"
    t, oc = synth.sparse_np(8192, M, seed=args.seed)
    if name == "dynamorio":
        oc[:] = 0
    # first, before this process touches the GPU: the loop from C (tools/plugin_loop.c)
    c_loop = plugin_loop_c(name, t, oc, M)
    torch.cuda.set_device(0)
    L = C.CDLL(build.PLUGIN_LIB)
    create = getattr(L, f"kbz_{name}_gpu_create")
    create.restype, create.argtypes = C.c_void_p, [C.c_char_p, C.c_char_p]
    record = getattr(L, f"kbz_{name}_gpu_record")
    record.restype, record.argtypes = C.c_long, [C.c_void_p, C.c_void_p, C.c_int]
    result = getattr(L, f"kbz_{name}_gpu_result")
    result.restype, result.argtypes = C.c_int, [C.c_void_p, C.c_long]
    cleanup = getattr(L, f"kbz_{name}_gpu_cleanup")
    cleanup.argtypes = [C.c_void_p]

    def per_exec(pool):
        """us per exec at each batch size; traces taken round-robin from the first `pool` rows"""
        per = {}
        for bs in (1, 16, 256, 4096):
            p = create(json.dumps({"map_size": M, "max_batch": bs}).encode(), None)
            if not p:
                raise SystemExit("plugin create failed")
            total = 1024 if bs == 1 else 8192
            for j in range(min(bs, 64)):  # warm: context, pinned slots
                result(p, record(p, t[j % pool].ctypes.data, int(oc[j % pool])))
            t0 = time.perf_counter()
            done = 0
            while done < total:
                k = min(bs, total - done)
                tickets = [record(p, t[(done + j) % pool].ctypes.data, int(oc[(done + j) % pool]))
                           for j in range(k)]
                for tk in tickets:
                    if result(p, tk) < 0:
                        raise SystemExit("plugin result failed")
                done += k
            el = time.perf_counter() - t0
            per[str(bs)] = round(1e6 * el / total, 3)
            cleanup(p)
        return per

    # cold: 8,192 distinct traces (512 MiB), every record copies from DRAM; hot: 16 traces (1 MiB)
    # cycled, the record copies from cache as it does from the target's just-written shm map
    per = per_exec(8192)
    per_hot = per_exec(16)
    by_c = {b: v["plugin_us"] for b, v in c_loop["by_batch"].items()}
    res = {"metric": "per-exec triage latency through the instrumentation plugin",
           "value": by_c["1"], "unit": "us/exec", "n_gpus": 1, "steps": 1, "warmup": 1,
           "higher_is_better": False, "vs_baseline": None, "dtype": "u8",
           "data": "synthetic config-2 traces in host memory",
           "config": {"workload": f"plugin {name}_gpu: record + result per exec from C in the "
                                  "fuzz loop's shape, batch sizes 1/16/256/4096",
                      "map_size": M, "mode": args.mode},
           "us_per_exec_by_batch": by_c,
           "c_loop": c_loop,
           "c_loop_note": "tools/plugin_loop.c: per exec memset(map) + the target's write of its "
                          "trace into a SysV shm map + record; every B execs result() for the B "
                          "tickets.  us_per_exec_by_batch = plugin_us = loop - the same loop "
                          "without the two plugin calls (base_us, timed after each loop)",
           "python_us_per_exec_by_batch": per,
           "python_us_per_exec_by_batch_hot_source": per_hot,
           "python_note": "the same calls through ctypes from Python (two foreign calls per exec "
                          "included): each record copies a trace from a 512 MiB pool "
                          "(DRAM-cold); _hot_source: 16 traces cycled"}
    if not args.no_cpu:
        cb = cpu_baseline(torch.from_numpy(t), torch.from_numpy(oc),
                          1 if name == "dynamorio" else 0, min(args.cpu_seconds, 5.0))
        cb["us_per_exec"] = round(1e6 / cb["value"], 3)
        res["cpu_baseline"] = cb
    print(json.dumps(res), flush=True)


def profile_first(args):
    """The profiler children of a one-GPU run (rank 0), started before this process touches the
    GPU: the kernel trace and the PMC passes of config 2 / 3, the PMC passes of the merge fold.
    Failures are reported in the line, never fatal."""
    pre = {"traffic": None, "ktrace": None, "valu": None}
    if args.gpus != 1 or os.environ.get("WORLD_SIZE", "1") != "1":
        return pre
    if args.workload in ("config2", "config3"):
        if args.ktrace:
            try:
                pre["ktrace"] = live_kernel_trace(args, steps=min(args.steps, 12))
            except Exception as e:  # noqa: BLE001
                pre["ktrace"] = {"avg_ms": None,
                                 "what": f"kernel trace failed: {type(e).__name__}: {e}"[:300]}
        if args.pmc:
            try:
                pre["traffic"] = live_traffic(args)
            except Exception as e:  # noqa: BLE001
                pre["traffic"] = {"bytes": None, "source": f"live PMC failed: {type(e).__name__}"}
            if args.workload == "config3":
                try:
                    pre["valu"] = live_valu(args)
                except Exception as e:  # noqa: BLE001
                    pre["valu"] = {"instructions_per_launch": None,
                                   "what": f"live PMC failed: {type(e).__name__}"}
    elif args.workload == "merge" and args.pmc:
        try:
            pre["traffic"] = merge_traffic(args)
        except Exception as e:  # noqa: BLE001
            pre["traffic"] = {"bytes": None, "source": f"live PMC failed: {type(e).__name__}"}
    return pre


def main():
    args = parse()
    maybe_launch(args)
    pre = profile_first(args)  # before any GPU call in this process
    {"merge": main_merge, "stream": main_stream, "plugin": main_plugin}.get(
        args.workload, main_triage)(args, pre)


if __name__ == "__main__":
    main()
