import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "convolutional-codes_amd")
for p in (PKG_ROOT, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def golden_manifest(kind="viterbi"):
    name = "manifest.json" if kind == "viterbi" else f"manifest_{kind}.json"
    with open(os.path.join(REPO, "tests", "golden", name)) as f:
        return json.load(f)


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """Bring the in-tree libraries up to date (hipcc cross-compiles without a GPU). make is
    incremental: a no-op on an up-to-date tree, a rebuild of exactly the stale libraries otherwise,
    so stale or missing shims are never tested."""
    import subprocess
    subprocess.run(["make", "-C", PKG_ROOT, "-j8"], check=True, capture_output=True)
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True,
                   capture_output=True)
