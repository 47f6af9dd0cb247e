#!/usr/bin/env python3
"""CFG-aware static check for kernels that issue VMEM loads from inline asm (k_pass1s).

The compiler does not know an asm `global_load` is still in flight, so it may copy, reuse or
overwrite its destination registers before the hand-written `s_waitcnt vmcnt(N)`.  This walks
the ISA of each kernel as a control-flow graph (labels / s_branch / s_cbranch_*), models vmcnt
as an in-order queue of VMEM ops (loads, stores, atomics; youngest first), joins queues at
merge points (element-wise union, aligned at the youngest op: vmcnt(N) keeps the N youngest)
and iterates to a fixpoint.  It reports every instruction that reads or writes a VGPR whose
load may still be pending.  Not part of the product (build-time check, tests/test_hazards.py).

usage: vmem_hazard_cfg.py file.s [kernel-substring]
"""
import re
import sys

VMEM_LOAD = ("global_load", "buffer_load", "flat_load", "scratch_load")
VMEM_STORE = ("global_store", "global_atomic", "buffer_store", "buffer_atomic", "flat_store",
              "flat_atomic", "scratch_store")
QMAX = 64


def regs(tok):
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def split_functions(lines):
    funcs, cur = {}, None
    for l in lines:
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            funcs[cur].append(l)
            if l.strip().startswith(".Lfunc_end"):
                cur = None
    return funcs


def blocks(body):
    """-> list of (label, [(lineno, text)]), successor map."""
    bl, cur = [], ("<entry>", [])
    for i, l in enumerate(body):
        t = l.split(";")[0].strip()
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            bl.append(cur)
            cur = (m.group(1), [])
            continue
        if not t or t.startswith("."):
            continue
        cur[1].append((i + 1, t))
    bl.append(cur)
    # split blocks after branches so every block ends in at most one branch
    out = []
    for lab, ins in bl:
        part, k = [], 0
        for x in ins:
            part.append(x)
            op = x[1].split()[0]
            if op.startswith("s_cbranch") or op == "s_branch" or op == "s_endpgm":
                out.append((lab if k == 0 else f"{lab}#{k}", part))
                part, k = [], k + 1
        if part or k == 0:
            out.append((lab if k == 0 else f"{lab}#{k}", part))
    succ = {}
    for idx, (lab, ins) in enumerate(out):
        nxt = out[idx + 1][0] if idx + 1 < len(out) else None
        s = []
        last = ins[-1][1] if ins else ""
        op = last.split()[0] if last else ""
        if op == "s_branch":
            s.append(last.split()[1])
        elif op.startswith("s_cbranch"):
            s.append(last.split()[1])
            if nxt:
                s.append(nxt)
        elif op == "s_endpgm":
            pass
        elif nxt:
            s.append(nxt)
        succ[lab] = s
    return out, succ


def join(a, b):
    if a is None:
        return list(b)
    n = max(len(a), len(b))
    r = []
    for i in range(n):
        x = a[i] if i < len(a) else set()
        y = b[i] if i < len(b) else set()
        r.append(x | y)
    return r[:QMAX]


def step(q, t, issues=None, where=None):
    """Apply one instruction to queue q (youngest first); record hazards."""
    op = t.split()[0]
    ops = [o.strip() for o in t[len(op):].split(",")]
    if op.startswith("s_waitcnt"):
        m = re.search(r"vmcnt\((\d+)\)", t)
        if m:
            q = q[: int(m.group(1))]
        return q
    pend = set().union(*q) if q else set()
    if op.startswith(VMEM_LOAD) and ("_lds_" in op or " lds" in t):
        # LDS-DMA (global_load_lds_dwordx4 vaddr, ...): no VGPR destination, the data goes to
        # LDS at M0; every VGPR operand is an address source
        srcs = set().union(*[regs(o) for o in ops]) if ops else set()
        if issues is not None and srcs & pend:
            issues.append((where, t, "address reads pending", sorted(srcs & pend)))
        return ([set()] + q)[:QMAX]
    if op.startswith(VMEM_LOAD):
        srcs = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        if issues is not None and srcs & pend:
            issues.append((where, t, "address reads pending", sorted(srcs & pend)))
        return ([regs(ops[0])] + q)[:QMAX]
    if op.startswith(VMEM_STORE):
        srcs = set().union(*[regs(o) for o in ops]) if ops else set()
        if issues is not None and srcs & pend:
            issues.append((where, t, "store reads pending", sorted(srcs & pend)))
        return ([set()] + q)[:QMAX]
    if op.startswith(("v_", "ds_", "s_")):
        touched = set().union(*[regs(o) for o in ops]) if ops else set()
        if issues is not None and touched & pend:
            issues.append((where, t, "touches pending", sorted(touched & pend)))
    return q


def scan_function(body):
    bl, succ = blocks(body)
    index = {lab: i for i, (lab, _) in enumerate(bl)}
    entry_state = {bl[0][0]: []}
    work = [bl[0][0]]
    while work:
        lab = work.pop()
        q = entry_state[lab]
        for _, t in bl[index[lab]][1]:
            q = step(q, t)
        for s in succ.get(lab, []):
            if s not in index:
                continue
            new = join(entry_state.get(s), q)
            if entry_state.get(s) != new:
                entry_state[s] = new
                work.append(s)
    issues = []
    for lab, ins in bl:
        q = entry_state.get(lab)
        if q is None:
            continue
        for ln, t in ins:
            q = step(q, t, issues, ln)
    return issues


def main():
    lines = open(sys.argv[1]).read().split("\n")
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_pass1s"
    total = 0
    for name, body in split_functions(lines).items():
        if sub not in name:
            continue
        iss = scan_function(body)
        total += len(iss)
        print(f"{name}: {len(iss)} potential hazards")
        for x in iss[:10]:
            print("   ", x)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
