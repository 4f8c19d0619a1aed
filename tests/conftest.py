import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def built():
    import __graft_entry__
    __graft_entry__.build()
    return True


@pytest.fixture(scope="session")
def zp(built):
    return importlib.import_module("zero-packet_amd")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "parse_golden.json")) as f:
        return json.load(f)
