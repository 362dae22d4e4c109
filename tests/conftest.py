import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmi_sim.so)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (and the HIP library when hipcc exists) once per session."""
    import __graft_entry__ as g

    g.build_oracle()
    if os.path.exists("/opt/rocm/bin/hipcc"):
        g.build_hip()
        g.build_rl()
    yield


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
