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
    """Build the in-tree libraries once if they are missing (hipcc cross-compiles without a GPU)."""
    import subprocess
    need = [os.path.join(PKG_ROOT, "lib", n) for n in
            ("libccv_core.so", "libccv_awgn.so", "libccv_bsc.so", "libccv_sim.so",
             "libccv_stack_awgn.so", "libccv_stack_bsc.so", "libccv_fano_awgn.so", "libccv_fano_bsc.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", PKG_ROOT, "-j8"], check=True, capture_output=True)
    if not os.path.exists(os.path.join(REPO, "oracle", "build", "libccoracle.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True,
                       capture_output=True)
