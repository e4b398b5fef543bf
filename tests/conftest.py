import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libwcb.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU test (minutes); runs with WCB_RUN_SLOW=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("WCB_RUN_SLOW") == "1":
        return
    skip = pytest.mark.skip(reason="slow CPU test: set WCB_RUN_SLOW=1 (tests/golden pin at full depth)")
    for it in items:
        if "slow" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
