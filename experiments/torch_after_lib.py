"""Diagnostic: does torch's HIP init still work after the library has run in the process?
usage: python torch_after_lib.py {ctx|ctx_nodestroy|odo|sr}"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "b-shot-slam_amd"))
import bshot_py  # noqa: E402

mode = sys.argv[1]
if mode in ("ctx", "ctx_nodestroy", "sr"):
    c = bshot_py.Context(0)
    if mode == "sr":
        pc, _ = bshot_py.synth_sweep(0)
        c.set_cloud(pc)
        c.seg_ratio()
    if mode != "ctx_nodestroy":
        c.close()
elif mode == "odo":
    o = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=256))
    pc, _ = bshot_py.synth_sweep(0)
    o.process(pc)
    o.close()
import torch  # noqa: E402

try:
    torch.zeros(1).cuda()
    print(mode, "torch ok", flush=True)
except Exception as e:  # noqa: BLE001
    print(mode, "torch FAILED:", e, flush=True)
