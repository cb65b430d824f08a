import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "mpc-ntm-control_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def ctl():
    """One NtmMpc controller (HIP library, device 0) per session."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ntm_mpc import NtmMpc
    c = NtmMpc()
    yield c
    c.close()
