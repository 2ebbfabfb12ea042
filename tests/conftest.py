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


@pytest.fixture(params=[1, 2], ids=["one_pass", "two_pass"])
def fill_passes(request, dev):
    """In-place fills in one pass (the generate tiles store the fields: the
    default up to 524 288 frames) and in two (generate, then a store pass or
    an engine store step): sccsum_set_fill_single_max, thread-local."""
    from seastar_amd import native

    lib = native.load()
    native.check(lib.sccsum_set_fill_single_max(1 << 30 if request.param == 1 else 0), "sccsum_set_fill_single_max")
    yield request.param
    native.check(lib.sccsum_set_fill_single_max(native.FILL_SINGLE_MAX), "sccsum_set_fill_single_max")
