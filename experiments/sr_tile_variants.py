"""Time SR variants on one synthetic HDL-64 sweep (wall time of ctx.seg_ratio(), min of 15 runs; under
rocprofv3 --kernel-trace, experiments/sr_trace.py splits the SR kernels' durations per variant)."""
import sys, time
import numpy as np
sys.path[:0] = ["b-shot-slam_amd"]
import bshot_py

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
c.set_cloud(pc)
ref = None
for opts in [dict(sr_tile=0), dict(sr_tile=1), dict(sr_tile=2), dict(sr_tile=3), dict(sr_tile=1, sr_tile_q=512),
             dict(sr_tile=2, sr_tile_q=1024), dict(sr_tile=0)] + [dict(sr_tile=int(a)) for a in sys.argv[1:]]:
    for k, v in opts.items():
        c.set_option(k, v)
    ts = []
    for _ in range(15):
        c.set_cloud(pc)
        t0 = time.perf_counter()
        idx, rat = c.seg_ratio()
        ts.append(time.perf_counter() - t0)
    same = ref is None or (np.array_equal(idx, ref[0]) and np.array_equal(rat.view(np.uint32), ref[1].view(np.uint32)))
    if ref is None:
        ref = (idx, rat)
    print(opts, f"min {min(ts) * 1e3:.3f} ms  median {np.median(ts) * 1e3:.3f} ms  same={same}", flush=True)
    c.set_option("sr_tile_q", 128)
c.close()
