import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def spark(tmp_path):
    """A fresh single-process session rooted in a temporary warehouse."""
    import cdnaml

    s = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(tmp_path / "warehouse")).getOrCreate()
    yield s
    s.stop()
