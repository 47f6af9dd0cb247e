"""Instruction mix of the loops of one kernel in a hipcc -S listing (not part of the product).

usage: python tools/isa_loops.py k.s <mangled-name substring> [--ops]
Each backward branch closes a loop; prints its label, length and VALU / SALU / LDS / VMEM
counts (and, with --ops, the VALU opcode histogram), so kernel variants can be compared by the
work their inner loops issue.
"""
import collections
import re
import sys


def function_body(lines, sub):
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m and sub in m.group(1):
            j = i
            while not lines[j].strip().startswith("s_endpgm"):
                j += 1
            return m.group(1), lines[i:j + 1]
    raise SystemExit(f"no function matching {sub}")


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    lines = open(sys.argv[1]).read().split("\n")
    name, body = function_body(lines, sys.argv[2])
    print(name, len(body), "lines")
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\S*\s+(\.LBB\S+)", l)
        if not m or labels.get(m.group(1), 1 << 30) >= i:
            continue
        c, ops = collections.Counter(), collections.Counter()
        for s in body[labels[m.group(1)]:i + 1]:
            s = s.strip()
            if not s or s.startswith((";", ".")):
                continue
            op = s.split()[0]
            c[kind(op)] += 1
            if op.startswith("v_"):
                ops[op] += 1
        print(f"loop {m.group(1)} lines {labels[m.group(1)]}-{i}: {dict(c)}")
        if "--ops" in sys.argv:
            for op, k in ops.most_common():
                print(f"    {k:5d} {op}")


if __name__ == "__main__":
    main()
