import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "b-shot-slam_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    # build the oracle (test infrastructure) and the product library if this checkout has none
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(os.path.join(PKG, "lib", "libbshot_amd.so")) or not os.path.exists(
            os.path.join(PKG, "lib", "libbshot_synth.so")):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])


@pytest.fixture(scope="session")
def sweep0():
    import bshot_py
    pc, pose = bshot_py.synth_sweep(0)
    return pc
