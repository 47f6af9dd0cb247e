import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: full-size case (minutes)")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import killerbeez_amd._lib as L

    L.lib()  # fails loudly if the HIP library is missing
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def product_isa(tmp_path_factory):
    """Device ISA of the product kbz_triage.hip (gfx950), compiled once per session (CPU)."""
    import subprocess

    from killerbeez_amd import build

    out = tmp_path_factory.mktemp("isa") / "kbz_triage.s"
    subprocess.check_call([build.hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17",
                           "--cuda-device-only", "-S", "-I", build.INC, "-I", build.CSRC,
                           build.HIP_SOURCES[0], "-o", str(out)], stderr=subprocess.DEVNULL)
    return out.read_text()
