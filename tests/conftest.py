"""Test configuration: paths, the ``gpu`` marker, and golden-fixture loaders.

sys.path order: the drop-in package directory (our ``rescheduling`` and ``rsk``),
then tests/stubs (the test-only ``kubernetes`` client), then the repo root (for
``oracle``).  /root/reference is never on the path here: tests compare against
the committed fixtures in tests/golden/.
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "kubernetes-rescheduling_amd")
for p in (REPO, os.path.join(REPO, "tests", "stubs"), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and librsk.so")


def load_golden(name):
    with open(os.path.join(GOLDEN, name), "r", encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def wm_golden():
    return load_golden("wm_snapshots.json")


@pytest.fixture(scope="session")
def edge_golden():
    return load_golden("edge_cases.json")


@pytest.fixture(scope="session")
def synth_golden():
    return load_golden("synth.json")


@pytest.fixture(scope="session")
def metrics_golden():
    return load_golden("metrics.json")
