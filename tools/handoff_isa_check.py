#!/usr/bin/env python3
"""Static check of the in-launch hand-offs (k_tail, k_fin, k_small's ticket, k_pass1s's look-back
word) on the compiled ISA.

The hand-offs follow MI355X_MICROARCH.md's valid forms (§ inter-workgroup visibility):
  * producer with plain payload stores: every storing wave `s_waitcnt vmcnt(0)`, `s_barrier`,
    one lane `buffer_wbl2 sc1` (release), `s_waitcnt vmcnt(0)` -- which the compiler may drop, so
    the source adds an asm one -- then the flag store `global_store_dword ... sc1`;
  * ticket (k_fin): every wave's atomics drained (`s_waitcnt vmcnt(0)`), `s_barrier`, then one
    lane's agent-scope `global_atomic_add` (returning);
  * consumer: `sc1` poll, `buffer_inv sc1` (acquire), `s_waitcnt vmcnt(0)`, `s_barrier`.
This walks each kernel's instructions in layout order (conservative: a store laid out on another
path still counts as pending) and reports:
  - a flag store (`global_store_dword` with `sc1`) issued while an earlier VMEM write
    (store / atomic / `buffer_wbl2`) may be in flight -- the flag could overtake its payload;
  - a `buffer_wbl2` not followed by `s_waitcnt vmcnt(0)` before the next VMEM operation;
  - a returning `global_atomic_add` (ticket) without a drain and a barrier since the last write;
  - a `buffer_inv sc1` not followed by `s_waitcnt vmcnt(0)` before the next `s_barrier`.
Not part of the product (tests/test_handoff_isa.py).
usage: handoff_isa_check.py file.s
"""
import re
import sys

WRITE = ("global_store", "global_atomic", "buffer_store", "buffer_atomic", "flat_store",
         "flat_atomic")
VMEM = WRITE + ("global_load", "buffer_load", "flat_load")


def split_functions(lines):
    funcs, cur = {}, None
    for line in lines:
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            s = line.split(";")[0].strip()
            if s and not s.startswith("."):
                funcs[cur].append(s)
    return funcs


def drains(ins):
    return ins.startswith("s_waitcnt") and re.search(r"vmcnt\(0\)", ins) is not None


def check(body, tickets=True, flags=True):
    """Returns (issues, counts) for one kernel body; tickets=False: returning atomic adds are
    list reservations (k_tail's item / fix-list appends), not signals; flags=False: the kernel's
    `sc1` dword stores re-arm words for the next launch (k_small), they signal nothing in-launch.
    A `buffer_wbl2` (release) waited for by `s_waitcnt vmcnt(0)` after the workgroup barrier
    keeps that barrier valid for a following ticket (k_small: drain, barrier, release, ticket)."""
    issues = []
    pending = False        # a VMEM write may be in flight
    payload = False        # ... of which a store / atomic (not only a release)
    barrier_after_drain = False
    wbl2_open = None       # index of a buffer_wbl2 not yet followed by vmcnt(0)
    inv_open = None        # index of a buffer_inv sc1 not yet followed by vmcnt(0)
    counts = {"flag_stores": 0, "wbl2": 0, "tickets": 0, "inv": 0}
    for i, ins in enumerate(body):
        op = ins.split()[0]
        if drains(ins):
            if payload:  # stores / atomics were in flight: a barrier must follow this drain
                barrier_after_drain = False
            pending = False
            payload = False
            wbl2_open = None
            inv_open = None
            continue
        if op == "s_barrier":
            if inv_open is not None:
                issues.append((inv_open, body[inv_open], "acquire not waited before the barrier"))
                inv_open = None
            if not pending:
                barrier_after_drain = True
            continue
        if op == "buffer_wbl2":
            counts["wbl2"] += 1
            wbl2_open = i
            pending = True
            continue
        if op == "buffer_inv":
            counts["inv"] += 1
            inv_open = i
            continue
        if op.startswith(VMEM):
            if wbl2_open is not None:
                issues.append((wbl2_open, body[wbl2_open], f"release not waited before {ins}"))
                wbl2_open = None
            is_flag = flags and op == "global_store_dword" and re.search(r"\bsc1\b", ins)
            is_ticket = tickets and op == "global_atomic_add" and re.search(r"\bsc0\b", ins)
            if is_flag:
                counts["flag_stores"] += 1
                if pending:
                    issues.append((i, ins, "flag store with a write still in flight"))
            if is_ticket:
                counts["tickets"] += 1
                if pending or not barrier_after_drain:
                    issues.append((i, ins, "ticket without drain + barrier"))
            if op.startswith(WRITE):
                pending = True
                payload = True
                barrier_after_drain = False
    return issues, counts


def lookback(body):
    """k_pass1s's in-launch look-back (the fused skip rule): the previous chunk's last-row hash
    travels with the batch tag in ONE 64-bit agent-scope word -- published by one
    `global_store_dwordx2 ... sc1`, polled by `global_load_dwordx2 ... sc1` -- so there is no
    payload to order it after.  Returns (publishes, polls, other sc1 stores)."""
    pub = [x for x in body if x.startswith("global_store_dwordx2") and re.search(r"\bsc1\b", x)]
    poll = [x for x in body if x.startswith("global_load_dwordx2") and re.search(r"\bsc1\b", x)]
    other = [x for x in body if x.startswith(("global_store", "buffer_store")) and
             re.search(r"\bsc1\b", x) and x not in pub]
    return pub, poll, other


def main():
    funcs = split_functions(open(sys.argv[1]).read().split("\n"))
    rc = 0
    for name, body in funcs.items():
        if "k_tail" not in name and "k_fin" not in name:
            continue
        issues, counts = check(body, tickets="k_fin" in name)
        print(name, counts, "OK" if not issues else issues[:5])
        rc |= bool(issues)
    return rc


if __name__ == "__main__":
    sys.exit(main())
