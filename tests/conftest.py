import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libppr_hip.so on the device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from approximated_personalized_pagerank_amd import build
    build.build()
    import oracle
    oracle.build()
