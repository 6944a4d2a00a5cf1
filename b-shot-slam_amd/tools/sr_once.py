"""Diagnostic: run the SR kernel a few times on one synthetic sweep (for rocprofv3 counter passes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
c.set_cloud(pc)
for _ in range(3):
    c.seg_ratio()
c.sync()
print("ok")
