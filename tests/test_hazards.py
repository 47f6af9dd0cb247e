"""Static check of pass 1's hand-counted VMEM waits (tools/vmem_hazard_cfg.py).

The pass-1 kernels (k_pass1s, the wide-map k_pass1w / k_pass1d and the no-hash k_pass1n) issue their prefetch loads from
inline asm, which the compiler does not track: it may copy, reuse or overwrite a destination
register before the hand-written `s_waitcnt vmcnt(N)`.  This compiles the device code to ISA,
walks every k_pass1s, k_pass1w, k_pass1d and k_pass1n instantiation as a control-flow graph with an in-order vmcnt
queue, and requires that no instruction touches a register whose load may still be in flight.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.parametrize("flags", [[], ["-DKBZ_ABLATION"]], ids=["product", "ablation"])
def test_pass1_has_no_inflight_register_hazards(tmp_path, flags, request):
    import vmem_hazard_cfg as V
    from killerbeez_amd import build

    if not flags:
        text = request.getfixturevalue("product_isa")
    else:
        out = tmp_path / "k.s"
        subprocess.check_call([build.hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17",
                               "--cuda-device-only", "-S", "-I", build.INC, "-I", build.CSRC,
                               *flags, build.HIP_SOURCES[0], "-o", str(out)],
                              stderr=subprocess.DEVNULL)
        text = out.read_text()
    funcs = V.split_functions(text.split("\n"))
    pass1 = {k: v for k, v in funcs.items()
             if any(p in k for p in ("k_pass1s", "k_pass1w", "k_pass1n", "k_pass1d"))}
    assert any("k_pass1s" in k for k in pass1), "no k_pass1s instantiation found in the ISA"
    if not flags:  # the ablation build compiles only k_pass1s
        assert sum("k_pass1w" in k for k in pass1) == 8, sorted(pass1)
        assert sum("k_pass1n" in k for k in pass1) == 4, sorted(pass1)
        assert sum("k_pass1d" in k for k in pass1) == 4, sorted(pass1)
    bad = {k: V.scan_function(v) for k, v in pass1.items()}
    bad = {k: v[:3] for k, v in bad.items() if v}
    assert not bad, bad


def test_checker_catches_a_reused_destination():
    """A register reused while its asm load is in flight must be reported."""
    import vmem_hazard_cfg as V

    body = ["global_load_dwordx4 v[2:5], v[0:1], off nt",
            "v_mov_b32_e32 v3, 0",
            "s_waitcnt vmcnt(0)",
            "s_endpgm"]
    assert V.scan_function(body)


def test_patprobe2_register_modes_are_hazard_free():
    """tools/patprobe2.hip (the staging calibration probe) with register-safe waits: no
    instruction touches a register whose asm load is in flight, in any instantiation -- round 5's
    plain-wait build of probe<0,256,3,0> faulted on the GPU (tools/patprobe2_hazards.py)."""
    import patprobe2_hazards as P

    out = []
    assert P.report(P.isa([]), "current", out) == 0, "\n".join(out)
