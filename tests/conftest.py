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
    # Build (incrementally) the oracle (test infrastructure) and the product library, so a local run
    # never tests a stale library. On the GPU box the tree arrives prebuilt without its object
    # files (b-shot-slam_amd/build is gpurun-ignored), so nothing is rebuilt there.
    libs = [os.path.join(PKG, "lib", n) for n in ("libbshot_amd.so", "libbshot_synth.so")]
    if os.environ.get("GRAFT_REPO_ROOT") or (not os.path.isdir(os.path.join(PKG, "build"))
                                             and all(os.path.exists(x) for x in libs)):
        return
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG])


@pytest.fixture(scope="session")
def sweep0():
    import bshot_py
    pc, pose = bshot_py.synth_sweep(0)
    return pc
