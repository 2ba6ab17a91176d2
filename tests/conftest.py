import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmsis-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the gpurun box)")
    config.addinivalue_line("markers", "slow: full-size property checks")


@pytest.fixture(scope="session")
def ref():
    """The reference scalar C path (oracle/_ref, built from /root/reference by oracle/ref.mk)."""
    import refs
    return refs.ref_lib()


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (oracle/_build/liboracle.so)."""
    import refs
    return refs.oracle_lib()


@pytest.fixture(scope="session")
def dsp():
    import cmsisdsp_amd
    return cmsisdsp_amd


@pytest.fixture(scope="session")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch
