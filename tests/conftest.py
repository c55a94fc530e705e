import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("FEDREC_QUIET", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built _C.so extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from fedrec_with_pytorchdistributed_amd.ops import native

    native.lib()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda", 0)
