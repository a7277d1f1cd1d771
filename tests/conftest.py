import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (HIP device); parity tests proper")


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(ROOT, "tests", "golden", name)) as f:
            return json.load(f)
    return load


@pytest.fixture
def default_stream_backlog():
    """Returns a function that queues ~20 ms of GPU work on torch's current
    stream (the legacy default stream): work the test queues after it on
    that stream is still pending when the library is called, so a library
    kernel that is not ordered after it sees the old bytes."""
    def queue():
        import torch
        try:
            torch.cuda._sleep(int(4e7))
        except (AttributeError, RuntimeError):
            big = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
            for i in range(100):
                big.fill_(i & 0xFF)
    return queue
