"""The C-ABI libraries load on a CPU-only host and export every symbol their headers declare
(no compute calls: those need a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from killerbeez_amd import _lib
from killerbeez_amd import build as kbuild


def _exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_hip_library_exports_header():
    L = _lib.lib()
    declared = _lib.header_functions()
    assert declared, "no functions parsed from include/kbz_triage.h"
    exported = _exported(kbuild.HIP_LIB)
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert {n for n, _, _ in _lib.SIGNATURES} == set(declared)
    assert L.kbz_abi_version() == _lib.ABI_VERSION


def test_hip_library_is_gfx950():
    # the fat binary embeds a gfx950 code object
    data = open(kbuild.HIP_LIB, "rb").read()
    assert b"gfx950" in data


def test_plugin_library_exports_header():
    kbuild.build_plugin()
    if not os.path.exists(kbuild.PLUGIN_LIB):
        pytest.skip("plugin not built")
    hdr = open(os.path.join(kbuild.INC, "kbz_plugin.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = sorted(set(re.findall(r"\b(kbz_afl_gpu_[a-z0-9_]+|kbz_dynamorio_gpu_[a-z0-9_]+|kbz_instrumentation_factory)\s*\(", hdr)))
    assert declared
    exported = _exported(kbuild.PLUGIN_LIB)
    assert not [f for f in declared if f not in exported]
    C.CDLL(kbuild.PLUGIN_LIB)


def test_plugin_layout_matches_reference_header(tmp_path):
    """tests/native/abi_layout.c: kbz_instrumentation_t against the reference's own
    instrumentation/instrumentation.h (offsets, member types, appended members)."""
    ref = "/root/reference/instrumentation"
    if not os.path.exists(os.path.join(ref, "instrumentation.h")):
        pytest.skip("reference tree absent")
    exe = tmp_path / "abi_layout"
    src = os.path.join(os.path.dirname(__file__), "native", "abi_layout.c")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-I", ref, "-I", kbuild.INC,
                           src, "-o", str(exe)])
    assert subprocess.call([str(exe)]) == 0


def test_product_library_has_no_experiment_flags():
    """The shipped libkbz_hip.so is the plain product build: kbz_build_flags() is empty (timing
    variants and diagnostics live only in build_variants/, and report their -D flags)."""
    L = C.CDLL(kbuild.HIP_LIB)
    L.kbz_build_flags.restype = C.c_char_p
    assert L.kbz_build_flags() == b""
    if not os.environ.get("KBZ_HIP_LIB"):
        assert _lib.lib().kbz_build_flags() == b""


def test_product_build_refuses_extra_flags(monkeypatch):
    monkeypatch.setenv("KBZ_HIPCC_FLAGS", "-DKBZ_STAMPS")
    with pytest.raises(kbuild.BuildError):
        kbuild.build_hip()


def test_build_is_redone_when_the_command_changes(tmp_path):
    """The stamp is a digest of the compile command and of every source: a different flag set
    makes the library stale even when no source is newer than it."""
    out = str(tmp_path / "lib.so")
    src = tmp_path / "a.c"
    src.write_text("int f(void) { return 1; }\n")
    cmd = ["gcc", "-shared", "-fPIC", str(src), "-o", out + ".tmp"]
    kbuild._run(out, cmd, [str(src)], False)
    assert kbuild._up_to_date(out, cmd, [str(src)])
    assert not kbuild._up_to_date(out, cmd + ["-DX=1"], [str(src)])
    src.write_text("int f(void) { return 2; }\n")
    assert not kbuild._up_to_date(out, cmd, [str(src)])


def test_variant_flags_are_checked():
    with pytest.raises(kbuild.BuildError):
        kbuild.build_variant("bad", ["-O0"])
    with pytest.raises(kbuild.BuildError):
        kbuild.build_variant("bad", ['-DX="y"'])
