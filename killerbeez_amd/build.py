"""Build libkbz_hip.so (gfx950) and libkbz_plugin.so in-tree with hipcc / gcc.

The product is the C-ABI shared library; the .so files are git-ignored but travel to the GPU
box with the repository snapshot (they are not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
HIP_LIB = os.path.join(PKG, "libkbz_hip.so")
PLUGIN_LIB = os.path.join(PKG, "libkbz_plugin.so")
ARCH = os.environ.get("KBZ_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = [os.path.join(CSRC, "kbz_triage.hip"), os.path.join(CSRC, "kbz_set.hip"),
               os.path.join(CSRC, "kbz_ipt.hip")]
HIP_HEADERS = [os.path.join(CSRC, "kbz_device.h"), os.path.join(INC, "kbz_triage.h")]
PLUGIN_SOURCES = [os.path.join(CSRC, "kbz_plugin.c")]
PLUGIN_HEADERS = [os.path.join(INC, "kbz_plugin.h"), os.path.join(INC, "kbz_triage.h")]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.sep not in c or os.path.exists(c):
            return c
    return "hipcc"


def build_hip(force: bool = False, verbose: bool = False) -> str:
    if force or _stale(HIP_LIB, HIP_SOURCES + HIP_HEADERS):
        extra = os.environ.get("KBZ_HIPCC_FLAGS", "").split()
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function", "-I", INC, "-I", CSRC, *extra, *HIP_SOURCES,
               "-o", HIP_LIB + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(HIP_LIB + ".tmp", HIP_LIB)
    return HIP_LIB


def build_plugin(force: bool = False, verbose: bool = False) -> str:
    if not all(os.path.exists(s) for s in PLUGIN_SOURCES):
        return ""
    if force or _stale(PLUGIN_LIB, PLUGIN_SOURCES + PLUGIN_HEADERS + [HIP_LIB]):
        cmd = ["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-std=gnu11", "-pthread", "-I", INC,
               *PLUGIN_SOURCES, "-L", PKG, "-lkbz_hip", "-Wl,-rpath,$ORIGIN",
               "-o", PLUGIN_LIB + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(PLUGIN_LIB + ".tmp", PLUGIN_LIB)
    return PLUGIN_LIB


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hip(force, verbose)
    build_plugin(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
