"""Diagnostic: repeated context create / SR / knn-stats / destroy (looks for a teardown hang)."""
import faulthandler
import os
import sys

faulthandler.dump_traceback_later(int(os.environ.get("HT_TIMEOUT", "60")), exit=True)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "b-shot-slam_amd"))
import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
reserve = int(sys.argv[1]) if len(sys.argv) > 1 else 32
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ladders = [int(x) for x in os.environ.get("HT_LADDERS", "2").split(",")]
for it in range(iters):
    c = bshot_py.Context(0)
    c.set_option("side_cu_reserve", reserve)
    c.set_option("ladder_grids", ladders[it % len(ladders)])
    c.set_cloud(pc)
    c.seg_ratio()
    c.iss()
    c.set_timing(True)
    c.stage_reset()
    c.set_cloud(pc)
    c.seg_ratio()
    c.stage_times()
    c.set_timing(False)
    c.knn_stats()
    print("iter", it, "closing", flush=True)
    c.close()
    print("iter", it, "ok", flush=True)
