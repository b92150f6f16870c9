"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on the CPU container (oracle vs golden fixtures, host
logic, C-ABI load/export checks, gloo multi-process paths); `-m gpu` runs the
parity tests proper on an MI355X through the C ABI.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "oracle"), os.path.join(REPO, "mitsuba-alvrl_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libalvrl.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu_ok():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return True
