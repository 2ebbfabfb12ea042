import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsccsum.so on cuda:0)")


@pytest.fixture(scope="session")
def dev():
    import torch

    from seastar_amd import native

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    native.check(native.load().sccsum_init(0), "sccsum_init")
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
