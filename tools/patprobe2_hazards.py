#!/usr/bin/env python3
"""Static check of tools/patprobe2.hip's register modes (not product; round-5 fault analysis).

Compiles the probe's device code twice -- with round 5's plain counted wait
(-DPATPROBE2_PLAIN_WAIT) and with the register-safe wait it uses now -- and runs
tools/vmem_hazard_cfg.py over every probe instantiation.  For the faulting round-5
configuration probe<0,256,3,0> it prints the instruction that writes an address into a register
whose asm load is still in flight, the wait that lets that load land on it, and the load that
then uses the register as its address.  Exit status 1 if the current build has any hazard.

usage: patprobe2_hazards.py [out.txt]
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import vmem_hazard_cfg as V  # noqa: E402


def isa(defines):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "p.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3",
                               "--cuda-device-only", "-S", *defines,
                               os.path.join(HERE, "patprobe2.hip"), "-o", out],
                              stderr=subprocess.DEVNULL)
        return open(out).read().split("\n")


def name(k):
    m = re.search(r"probeILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", k)
    return f"probe<{','.join(m.groups())}>" if m else k


def report(lines, title, out):
    funcs = V.split_functions(lines)
    total = 0
    out.append(f"== {title}")
    for k, body in sorted(funcs.items()):
        if "probe" not in k:
            continue
        iss = V.scan_function(body)
        total += len(iss)
        out.append(f"{name(k)}: {len(iss)} instructions touch a register whose load is in flight")
        # an address written into a pending register, then used by a load: the fault pattern
        for ln, t, kind, regs_ in iss:
            op = t.split()[0]
            dst = V.regs(t[len(op):].split(",")[0])
            if not (dst and dst <= set(regs_) and op.startswith("v_lshl_add_u64")):
                continue
            txt = [l.split(";")[0].strip() for l in body]
            use = next((j for j in range(ln, min(len(txt), ln + 40))
                        if txt[j].startswith("global_load") and
                        V.regs(txt[j].split(",")[1]) == dst), None)
            wait = next((j for j in range(ln, use or ln) if txt[j].startswith("s_waitcnt vmcnt")),
                        None)
            issue = next((j for j in range(ln - 2, -1, -1) if txt[j].startswith("global_load")
                          and V.regs(txt[j].split()[1].rstrip(",")) >= dst), None)
            if use is None:
                continue
            out.append(f"   in flight:  line {issue + 1}: {txt[issue]}" if issue is not None
                       else "   in flight:  (a load of an earlier iteration)")
            out.append(f"   clobber:    line {ln}: {t}")
            if wait is not None:
                out.append(f"   wait:       line {wait + 1}: {txt[wait]}  (lets that load land "
                           "on the address)")
            out.append(f"   faulting:   line {use + 1}: {txt[use]}")
    return total


def main():
    out = []
    report(isa(["-DPATPROBE2_PLAIN_WAIT"]), "round 5's plain s_waitcnt (PATPROBE2_PLAIN_WAIT)", out)
    bad = report(isa([]), "register-safe waits (the probe as built now)", out)
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(text + "\n")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
