import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cmt-cooperative-perception_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and the built libcmt_hip.so")


_PARITY = []


@pytest.fixture(scope="session")
def parity_log():
    """Tests append (case, measured max error, bound) lines; they are printed in
    the terminal summary so the run's tail carries the measured numbers."""
    return _PARITY


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if _PARITY:
        terminalreporter.write_sep("-", "measured parity (max abs error vs the oracle, bound)")
        for line in _PARITY:
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
