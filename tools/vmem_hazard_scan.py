#!/usr/bin/env python3
"""Static check for kernels that issue VMEM loads from inline asm (k_pass1s): walk the ISA of
one kernel in program order, model vmcnt as an in-order queue of VMEM ops (loads, stores,
atomics), retire on `s_waitcnt vmcnt(N)`, and report any VALU/SALU/DS instruction that writes
or reads a VGPR whose load is still pending.  Straight-line approximation: branches are
ignored (each basic block is assumed to follow the previous one in the listing), which is
conservative for the loop bodies checked here.

usage: vmem_hazard_scan.py kernel.s
"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return [int(m.group(1))] if m else []


def scan(lines):
    queue = []  # list of sets of destination regs (empty set for stores/atomics)
    issues = []
    for i, line in enumerate(lines):
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        ops = [o.strip() for o in t[len(op):].split(",")]
        if op.startswith("s_waitcnt"):
            m = re.search(r"vmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                while len(queue) > n:
                    queue.pop(0)
            continue
        pend = set().union(*queue) if queue else set()
        if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
            srcs = [r for o in ops[1:] for r in regs(o)]
            bad = [r for r in srcs if r in pend]
            if bad:
                issues.append((i + 1, t, "address reads pending", bad))
            queue.append(set(regs(ops[0])))
            continue
        if op.startswith(("global_store", "global_atomic", "buffer_store", "buffer_atomic")):
            srcs = [r for o in ops for r in regs(o)]
            bad = [r for r in srcs if r in pend]
            if bad:
                issues.append((i + 1, t, "store reads pending", bad))
            queue.append(set())
            continue
        touched = [r for o in ops for r in regs(o)]
        bad = [r for r in touched if r in pend]
        if bad and (op.startswith(("v_", "ds_", "s_"))):
            issues.append((i + 1, t, "touches pending", bad))
    return issues


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().split("\n")
    iss = scan(lines)
    for x in iss[:40]:
        print(x)
    print(f"{len(iss)} potential hazards")
    sys.exit(1 if iss else 0)
