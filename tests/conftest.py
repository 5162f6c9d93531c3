import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library on cuda:0)")


@pytest.fixture(scope="session")
def oracle():
    from oracle_bindings import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def ofdm():
    import ofdm_lsmrc
    ofdm_lsmrc.lib()
    return ofdm_lsmrc


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
