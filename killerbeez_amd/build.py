"""Build libkbz_hip.so (gfx950) and libkbz_plugin.so in-tree with hipcc / gcc.

The product is the C-ABI shared library; the .so files are git-ignored but travel to the GPU
box with the repository snapshot (they are not gpurun-ignored).

The product library is always built from the sources as they are, with no extra preprocessor
flags: `KBZ_HIPCC_FLAGS` is refused for it.  Experiment builds (timing A/Bs, the `KBZ_STAMPS`
cycle-stamp diagnostic) go to `build_variants/<name>/libkbz_hip.so` through `build_variant()`
(`python -m killerbeez_amd.build --variant NAME -DFLAG ...`) and report their flags through
`kbz_build_flags()`; the product reports "".  Each library carries a stamp file holding a
digest of its compile command and of every source and header: a build is redone when either
changes, not only when a source is newer than the library.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
HIP_LIB = os.path.join(PKG, "libkbz_hip.so")
PLUGIN_LIB = os.path.join(PKG, "libkbz_plugin.so")
VARIANTS = os.path.join(ROOT, "build_variants")
ARCH = os.environ.get("KBZ_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = [os.path.join(CSRC, "kbz_triage.hip"), os.path.join(CSRC, "kbz_set.hip"),
               os.path.join(CSRC, "kbz_ipt.hip"), os.path.join(CSRC, "kbz_multi.hip")]
HIP_HEADERS = [os.path.join(CSRC, "kbz_device.h"), os.path.join(INC, "kbz_triage.h")]
PLUGIN_SOURCES = [os.path.join(CSRC, "kbz_plugin.c")]
PLUGIN_HEADERS = [os.path.join(INC, "kbz_plugin.h"), os.path.join(INC, "kbz_triage.h")]


class BuildError(RuntimeError):
    pass


def _digest(cmd, deps) -> str:
    h = hashlib.sha256(" ".join(cmd).encode())
    for d in sorted(deps):
        h.update(d.encode())
        if os.path.exists(d):
            with open(d, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def _up_to_date(out, cmd, deps) -> bool:
    stamp = out + ".stamp"
    if not (os.path.exists(out) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == _digest(cmd, deps)


def _run(out, cmd, deps, verbose) -> None:
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    with open(out + ".stamp", "w") as f:
        f.write(_digest(cmd, deps) + "\n")


def hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.sep not in c or os.path.exists(c):
            return c
    return "hipcc"


def _hip_cmd(out, defines) -> list:
    # kbz_build_flags() reports the -D flags of a variant build (the product passes none)
    tag = " ".join(defines)
    return [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-Wall", "-Wno-unused-function", "-I", INC, "-I", CSRC, *defines,
            f"-DKBZ_BUILD_FLAGS_STR=\"{tag}\"", *HIP_SOURCES, "-ldl", "-o", out + ".tmp"]


def build_hip(force: bool = False, verbose: bool = False) -> str:
    if os.environ.get("KBZ_HIPCC_FLAGS", "").strip():
        raise BuildError("KBZ_HIPCC_FLAGS is not accepted for the product library; build "
                         "experiments with build_variant() into build_variants/<name>/")
    cmd = _hip_cmd(HIP_LIB, [])
    deps = HIP_SOURCES + HIP_HEADERS
    if force or not _up_to_date(HIP_LIB, cmd, deps):
        _run(HIP_LIB, cmd, deps, verbose)
    return HIP_LIB


def build_variant(name: str, defines, verbose: bool = False) -> str:
    """Experiment build: build_variants/<name>/libkbz_hip.so with extra -D flags.  Load it
    with KBZ_HIP_LIB=<path>; it never replaces the product library."""
    defines = list(defines)
    bad = [d for d in defines if not d.startswith("-D") or '"' in d]
    if bad or not name or os.sep in name:
        raise BuildError(f"variant flags must be -DNAME[=VALUE] without quotes: {bad}")
    out_dir = os.path.join(VARIANTS, name)
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "libkbz_hip.so")
    cmd = _hip_cmd(out, defines)
    deps = HIP_SOURCES + HIP_HEADERS
    if not _up_to_date(out, cmd, deps):
        _run(out, cmd, deps, verbose)
    return out


def build_plugin(force: bool = False, verbose: bool = False) -> str:
    if not all(os.path.exists(s) for s in PLUGIN_SOURCES):
        return ""
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-std=gnu11", "-pthread", "-I", INC,
           *PLUGIN_SOURCES, "-L", PKG, "-lkbz_hip", "-Wl,-rpath,$ORIGIN", "-lm",
           "-o", PLUGIN_LIB + ".tmp"]
    # the plugin links the product library: rebuilt when that changes too
    deps = PLUGIN_SOURCES + PLUGIN_HEADERS + [HIP_LIB + ".stamp"]
    if force or not _up_to_date(PLUGIN_LIB, cmd, deps):
        _run(PLUGIN_LIB, cmd, deps, verbose)
    return PLUGIN_LIB


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hip(force, verbose)
    build_plugin(force, verbose)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args[:1] == ["--variant"] and len(args) >= 2:
        print(build_variant(args[1], args[2:], verbose=True))
    else:
        build_all(force="--force" in args, verbose=True)
