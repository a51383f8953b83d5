import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zig-bpe_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libzbpe.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def gpu_available() -> bool:
    return os.path.exists("/dev/kfd")


@pytest.fixture(scope="session")
def engine():
    import zbpe

    e = zbpe.Engine(0)
    yield e
    e.close()
