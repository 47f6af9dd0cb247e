"""The branch-free byte transforms used by the gfx950 kernels (kbz_device.h) equal the
reference's byte lookup tables on every byte value and across byte boundaries."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.parametrize("cxx", ["g++", "/opt/rocm/llvm/bin/clang++"])
def test_swar_transforms_exhaustive(tmp_path, cxx):
    """g++ builds the portable bit reversal, clang the __builtin_bitreverse32 the kernels use."""
    if not os.path.exists(cxx) and cxx.startswith("/"):
        pytest.skip(f"{cxx} absent")
    exe = tmp_path / "swar_check"
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "killerbeez_amd", "csrc"),
                           os.path.join(HERE, "native", "swar_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "OK", out.stdout + out.stderr
