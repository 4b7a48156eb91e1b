import contextlib
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


# Every session-based test runs on the host ("cpu", the CPU suite) and on the GPU ("cuda", marked gpu: the
# MI355X suite selects it with -m gpu), so the course flows exercise the device kernels on hardware too.
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@contextlib.contextmanager
def session_device(device):
    """Sessions created inside use ``device`` (cpu / cuda; cuda skips without a GPU)."""
    import torch

    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = os.environ.get("CDNAML_DEVICE")
    os.environ["CDNAML_DEVICE"] = device
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("CDNAML_DEVICE", None)
        else:
            os.environ["CDNAML_DEVICE"] = old


@pytest.fixture(params=DEVICES)
def spark(request, tmp_path):
    """A fresh single-process session rooted in a temporary warehouse, on the parametrised device."""
    import cdnaml

    with session_device(request.param):
        s = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(tmp_path / "warehouse")).getOrCreate()
        assert s.device.type == request.param
        yield s
        s.stop()
