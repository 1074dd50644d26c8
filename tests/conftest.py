import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "sonido-sonar_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the GPU)")


@pytest.fixture(scope="session")
def ctx():
    import sonar
    c = sonar.Context(0)
    yield c
    c.close()
