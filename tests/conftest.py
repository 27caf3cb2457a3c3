import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("MPLBACKEND", "Agg")
GOLDEN = os.path.join(REPO, "tests", "golden")
TERMINAL_SETS = os.path.join(REPO, "terminal_sets")
CONFIGS = [("RoadEnv", 10), ("RoadEnv", 20), ("RoadOneCarEnv", 20), ("RoadMultipleCarsEnv", 20)]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the built HIP library")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
