"""Diagnostic: bench.py with one odometry parameter overridden (e.g. run_iss=0: how much of the period
ISS costs). Results are not product numbers. usage: python diag_param.py name=value [bench args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "b-shot-slam_amd"))
sys.path.insert(0, ROOT)
import bshot_py  # noqa: E402

name, value = sys.argv[1].split("=")
_orig = bshot_py.default_params


def _patched(**kw):
    p = _orig(**kw)
    setattr(p, name, int(value))
    return p


bshot_py.default_params = _patched
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
