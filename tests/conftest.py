import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def oracle():
    from hpmpc_amd.build import build_oracle
    from hpmpc_amd.cabi import HpmpcAPI, load

    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        build_oracle()
    return HpmpcAPI(load(path), "orc_")


@pytest.fixture(scope="session")
def product():
    """The HIP library through its reference-named C ABI (GPU tests only)."""
    import torch

    from hpmpc_amd.batch import LIBPATH
    from hpmpc_amd.cabi import HpmpcAPI, load

    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    return HpmpcAPI(load(LIBPATH), "")
