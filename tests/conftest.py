import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    """The built extension; on a GPU box a missing build is an error, not a skip."""
    from mikmeans.ops import native as nat

    return nat.require()


@pytest.fixture
def kvariant(native):
    """Set kernel A/B switches for one test (mikmeans.ops.native.set_variant), restored after."""
    from mikmeans.ops import native as nat

    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = nat.get_variant(name)
        nat.set_variant(name, int(value))

    yield set_
    for k, v in saved.items():
        nat.set_variant(k, v)
