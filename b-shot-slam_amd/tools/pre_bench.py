"""Preprocessor timing (diagnostics): device lasers -> device points, per-call wall ms and the
BSHOT_STAGE_PRE event time, for the synthetic sensors. Usage: python tools/pre_bench.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bshot_py  # noqa: E402
import torch  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = bshot_py.Context(0)
for sensor in (2, 0, 1):
    L = bshot_py.synth_lasers(0, sensor=sensor)
    v = bshot_py.sensor_vertical_angles(sensor)
    dl = torch.from_numpy(L.view(np.uint8)).cuda()
    out = torch.zeros((len(L), 3), dtype=torch.float32, device="cuda")
    for _ in range(3):
        n = ctx.preprocess_device(dl.data_ptr(), len(L), v, out.data_ptr(), len(L), lowpt_th=-1950.0)
    ctx.set_timing(True)
    ctx.stage_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        n = ctx.preprocess_device(dl.data_ptr(), len(L), v, out.data_ptr(), len(L), lowpt_th=-1950.0)
    el = (time.perf_counter() - t0) / reps * 1e3
    st = ctx.stage_times()["preprocess"]
    ctx.set_timing(False)
    print(f"sensor {sensor}: {len(L)} lasers -> {n} pts, wall {el:.3f} ms/call, device {st[0] / reps:.3f} ms/call "
          f"({st[1] // reps} timed segments)")
ctx.close()
