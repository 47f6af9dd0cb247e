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
# bench harness (not product): the plugins driven from C in the fuzz loop's shape
PLUGIN_LOOP = os.path.join(ROOT, "tools", "plugin_loop")
PLUGIN_LOOP_SRC = os.path.join(ROOT, "tools", "plugin_loop.c")


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


def _hip_cmd(out, defines, csrc=CSRC, tag_extra="") -> list:
    # kbz_build_flags() reports the -D flags (and patch) of a variant build (the product: "")
    tag = " ".join(defines) + tag_extra
    sources = [os.path.join(csrc, os.path.basename(f)) for f in HIP_SOURCES]
    return [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-Wall", "-Wno-unused-function", "-I", INC, "-I", csrc, *defines,
            f"-DKBZ_BUILD_FLAGS_STR=\"{tag}\"", *sources, "-ldl", "-o", out + ".tmp"]


def build_hip(force: bool = False, verbose: bool = False) -> str:
    if os.environ.get("KBZ_HIPCC_FLAGS", "").strip():
        raise BuildError("KBZ_HIPCC_FLAGS is not accepted for the product library; build "
                         "experiments with build_variant() into build_variants/<name>/")
    cmd = _hip_cmd(HIP_LIB, [])
    deps = HIP_SOURCES + HIP_HEADERS
    if force or not _up_to_date(HIP_LIB, cmd, deps):
        _run(HIP_LIB, cmd, deps, verbose)
    return HIP_LIB


def build_variant(name: str, defines, verbose: bool = False, patch: str | None = None) -> str:
    """Experiment build: build_variants/<name>/libkbz_hip.so with extra -D flags.  Load it
    with KBZ_HIP_LIB=<path>; it never replaces the product library.  `patch` (a unified diff
    against csrc/, e.g. tools/ab_p1s.patch: timing-only ablations with wrong results) is applied
    to a copy of the sources in build_variants/<name>/csrc -- such code never enters the
    product tree."""
    defines = list(defines)
    bad = [d for d in defines if not d.startswith("-D") or '"' in d]
    if bad or not name or os.sep in name:
        raise BuildError(f"variant flags must be -DNAME[=VALUE] without quotes: {bad}")
    out_dir = os.path.join(VARIANTS, name)
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "libkbz_hip.so")
    csrc, extra = CSRC, ""
    if patch:
        import shutil

        csrc = os.path.join(out_dir, "csrc")
        shutil.rmtree(csrc, ignore_errors=True)
        shutil.copytree(CSRC, csrc, ignore=shutil.ignore_patterns("*.so*", "__pycache__"))
        with open(patch) as f:
            subprocess.check_call(["patch", "-s", "-p1", "-d", csrc], stdin=f)
        extra = f" patch={os.path.basename(patch)}"
    cmd = _hip_cmd(out, defines, csrc, extra)
    deps = HIP_SOURCES + HIP_HEADERS + ([patch] if patch else [])
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


def build_plugin_loop(force: bool = False, verbose: bool = False) -> str:
    if not os.path.exists(PLUGIN_LOOP_SRC):
        return ""
    cmd = ["gcc", "-O2", "-Wall", "-std=gnu11", "-I", INC, PLUGIN_LOOP_SRC, "-L", PKG,
           "-lkbz_plugin", "-Wl,-rpath,$ORIGIN/../killerbeez_amd", "-o", PLUGIN_LOOP + ".tmp"]
    deps = [PLUGIN_LOOP_SRC, os.path.join(INC, "kbz_plugin.h"), PLUGIN_LIB + ".stamp"]
    if force or not _up_to_date(PLUGIN_LOOP, cmd, deps):
        _run(PLUGIN_LOOP, cmd, deps, verbose)
    return PLUGIN_LOOP


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hip(force, verbose)
    build_plugin(force, verbose)
    build_plugin_loop(force, verbose)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args[:1] == ["--variant"] and len(args) >= 2:
        rest, patch = args[2:], None
        if rest[:1] == ["--patch"] and len(rest) >= 2:
            patch, rest = os.path.abspath(rest[1]), rest[2:]
        print(build_variant(args[1], rest, verbose=True, patch=patch))
    else:
        build_all(force="--force" in args, verbose=True)
