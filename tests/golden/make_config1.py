#!/usr/bin/env python3
"""Generate tests/golden/config1.npz -- BASELINE config 1's golden trace dump: REAL traces of the
reference's own afl-gcc instrumentation on corpus/afl_test, with expected results from the
reference's own bitmap code.

1. afl-gcc and afl-as are compiled with gcc straight from /root/reference/afl_progs/afl-gcc.c
   and afl-as.c (flags of afl_progs/Makefile; no reference build system, nothing copied), into a
   temporary directory outside the repository.
2. corpus/afl_test/test.c is compiled with that afl-gcc (AFL_PATH = the temp dir, so its `as`
   is afl-as): the classic AFL trampoline writing map[cur ^ prev]++ (afl_progs/afl-as.h) into
   SysV SHM.  Edge IDs are random per build (afl-as.c seeds from time and pid), which is why the
   traces are captured once and committed; the target's sha256 is stored with them.
3. tests/golden/config1_runner.c (ours) runs the target once per input on stdin with a cleared
   SHM map and keeps the raw counters and the outcome (exit / timeout / signal).
4. Inputs: the bit-flip schedule "exec j flips bit j mod 32 of the seed" (the bit_flip mutator
   lives in the absent killerbeez-mutators, so its exact schedule is parity-unpinned; this is
   the schedule SURVEY.md §8(d) / VERDICT r1 name) over two seeds of tests/smoke_test.sh:
   "AAAA\\n" (config 1: 1,000 execs, `fuzzer stdin afl bit_flip -n 1000`) and "ABC@\\n" (100
   execs; exec 26 turns it into "ABCD", the NULL write: the crash the smoke test expects).
5. Expected results per sequence, each a fresh fuzzing run (virgin maps all 0xff), from
   oracle/_ref (the reference's own has_new_bits / simplify_trace / classify_counts / hash32,
   composed like finish_fuzz_round afl_instrumentation.c:231-274 and has_new_coverage
   dynamorio_instrumentation.c:1428-1468; see make_golden.ref_loop): per-exec hnb, hash32 and
   XXH64 for the afl and dynamorio modes, the final virgin maps and last hash.

Sanity (not parity): tests/smoke_test.sh:139-145 expects "Found new_paths" 2 times for `-n 10`
from "AAAA"; the count here is hnb != 0 among the first 10 AFL execs (stored as smoke_new_paths).

Run from the repository root (needs /root/reference):  python tests/golden/make_config1.py
"""
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import oracle  # noqa: E402
from make_golden import ref_loop, sparse  # noqa: E402

REF = "/root/reference"
M = 65536
CFLAGS = ["-O3", "-funroll-loops", "-Wall", "-D_FORTIFY_SOURCE=2", "-g", "-Wno-pointer-sign"]


def build(tmp):
    defs = [f'-DAFL_PATH="{tmp}"', f'-DDOC_PATH="{tmp}"', f'-DBIN_PATH="{tmp}"']
    for prog in ("afl-gcc", "afl-as"):
        subprocess.check_call(["gcc", *CFLAGS, *defs, f"{REF}/afl_progs/{prog}.c", "-o",
                               os.path.join(tmp, prog)])
    os.symlink("afl-as", os.path.join(tmp, "as"))
    env = dict(os.environ, AFL_PATH=tmp, AFL_QUIET="1")
    target = os.path.join(tmp, "afl_test")
    subprocess.check_call([os.path.join(tmp, "afl-gcc"), f"{REF}/corpus/afl_test/test.c", "-o",
                           target], env=env, stderr=subprocess.DEVNULL)
    runner = os.path.join(tmp, "runner")
    subprocess.check_call(["gcc", "-O2", "-Wall", os.path.join(HERE, "config1_runner.c"), "-o",
                           runner])
    return target, runner


def bitflip_inputs(seed: bytes, n: int):
    out = np.frombuffer(seed, np.uint8)[None].repeat(n, 0).copy()
    for j in range(n):
        b = j % 32
        out[j, b // 8] ^= np.uint8(1 << (b % 8))
    return out


def run(runner, target, inputs, tmp, tag):
    fi, fm, fo = (os.path.join(tmp, f"{tag}.{x}") for x in ("in", "maps", "oc"))
    inputs.tofile(fi)
    subprocess.check_call([runner, target, fi, str(inputs.shape[0]), str(inputs.shape[1]), fm, fo])
    maps = np.fromfile(fm, np.uint8).reshape(-1, M)
    oc = np.fromfile(fo, np.int8)
    assert maps.shape[0] == inputs.shape[0] == oc.shape[0]
    return maps, oc


def main():
    oracle.build()
    R = oracle.ref()
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        target, runner = build(tmp)
        out["target_sha256"] = np.frombuffer(
            hashlib.sha256(open(target, "rb").read()).hexdigest().encode(), np.uint8)
        for tag, seed, n in (("aaaa", b"AAAA\n", 1000), ("abc", b"ABC@\n", 100)):
            inputs = bitflip_inputs(seed, n)
            maps, oc = run(runner, target, inputs, tmp, tag)
            out[f"{tag}_inputs"] = inputs
            out[f"{tag}_n"] = np.array(n)
            out[f"{tag}_tj"], out[f"{tag}_ti"], out[f"{tag}_tv"] = sparse(maps)
            out[f"{tag}_outcome"] = oc
            for name, mode in (("afl", oracle.MODE_AFL), ("dynamorio", oracle.MODE_DYNAMORIO)):
                hnb, h32, x64, V, last = ref_loop(R, mode, maps, oc)
                out[f"{tag}_{name}_hnb"], out[f"{tag}_{name}_h32"] = hnb, h32
                out[f"{tag}_{name}_x64"] = x64
                vm, vi = np.nonzero(V != 0xFF)
                out[f"{tag}_{name}_vmap"], out[f"{tag}_{name}_vidx"] = vm.astype(np.uint8), vi.astype(np.uint32)
                out[f"{tag}_{name}_vval"] = V[vm, vi]
                out[f"{tag}_{name}_last"] = np.array(last, np.uint32)
            print(f"{tag}: {n} execs, {len(np.unique(maps, axis=0))} distinct traces, "
                  f"outcomes {np.bincount(oc, minlength=3).tolist()}, afl new paths "
                  f"{int((out[f'{tag}_afl_hnb'] > 0).sum())}, first 10: "
                  f"{int((out[f'{tag}_afl_hnb'][:10] > 0).sum())}")
        out["smoke_new_paths"] = np.array(int((out["aaaa_afl_hnb"][:10] > 0).sum()))
    np.savez_compressed(os.path.join(HERE, "config1.npz"), **out)


if __name__ == "__main__":
    main()
