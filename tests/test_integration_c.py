"""INTEGRATION.md's C patches compiled and run (tests/native/integration_harness.c): the factory
branch that copies the afl_gpu vtable into the reference's own instrumentation_t
(instrumentation_factory.c:72-84), and the patched finish_fuzz_round / afl_is_new_path
(afl_instrumentation.c:189-198, :231-274) driven like fuzzer/main.c:370-418 -- per exec, and
batched -- over BASELINE config 1's real afl-gcc traces (tests/golden/config1.npz, expected
results from the reference's own code)."""
import os
import subprocess

import numpy as np
import pytest

from killerbeez_amd import build as kbuild

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "integration_harness.c")
OUT = os.path.join(HERE, "native", "_build")
REF_INC = "/root/reference/instrumentation"


def build_harness(with_reference: bool | None = None) -> str:
    """Compile the harness (against the reference's instrumentation.h when that tree exists);
    the binary lands in tests/native/_build/ (git-ignored; it travels to the GPU box)."""
    if with_reference is None:
        with_reference = os.path.exists(os.path.join(REF_INC, "instrumentation.h"))
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "integration_harness" + ("" if with_reference else "_noref"))
    kbuild.build_plugin()
    flags = ["-I", REF_INC] if with_reference else ["-DKBZ_NO_REFERENCE_HEADER"]
    subprocess.check_call(["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", *flags, "-I",
                           kbuild.INC, SRC, "-L", kbuild.PKG, "-lkbz_plugin",
                           f"-Wl,-rpath,{kbuild.PKG}", "-o", exe])
    return exe


def test_harness_compiles_against_reference_header():
    if not os.path.exists(os.path.join(REF_INC, "instrumentation.h")):
        pytest.skip("reference tree absent")
    assert os.path.exists(build_harness(True))


def test_harness_compiles_without_reference_header():
    assert os.path.exists(build_harness(False))


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 7, 64])
def test_patched_afl_plugin_on_config1(gpu, batch, tmp_path):
    exe = os.path.join(OUT, "integration_harness")
    if not os.path.exists(exe):  # the box has no reference tree: the prebuilt binary travels
        exe = build_harness(False)
    f = np.load(os.path.join(HERE, "golden", "config1.npz"))
    for tag in ("abc", "aaaa"):
        n = min(int(f[f"{tag}_n"]), 300)
        t = np.zeros((int(f[f"{tag}_n"]), 65536), np.uint8)
        t[f[f"{tag}_tj"], f[f"{tag}_ti"]] = f[f"{tag}_tv"]
        oc = f[f"{tag}_outcome"].astype(np.int8)
        exp = f[f"{tag}_afl_hnb"]
        p = tmp_path / f"{tag}.bin"
        p.write_bytes(t[:n].tobytes() + oc[:n].tobytes())
        r = subprocess.run([exe, str(p), str(n), "65536", str(batch)], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.split("\n")
        got = np.array([int(l.split()[1]) for l in lines if l and not l.startswith("state")])
        np.testing.assert_array_equal(got, (exp[:n] != 0).astype(int), err_msg=f"{tag} batch {batch}")
        assert any(l.startswith("state ") for l in lines)
