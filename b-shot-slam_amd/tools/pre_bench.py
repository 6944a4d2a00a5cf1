"""Preprocessor and packet-decode timing (diagnostics; profiles/*_preprocess_*): device lasers ->
device points per synthetic sensor, and HDL-32E packet decode, with wall ms per call, the
BSHOT_STAGE_PRE event time and the achieved bytes/s of the decode (1206 B in + 384 x 32 B out per
packet). Usage: python tools/pre_bench.py [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bshot_py  # noqa: E402
import torch  # noqa: E402


def hdl32_packets(frames):
    """HDL-32E data packets carrying synth_lasers(sensor=2) rotations (12 firings x 32 returns)."""
    L = np.concatenate([bshot_py.synth_lasers(f, sensor=2) for f in frames])
    fir = L.reshape(-1, 32)
    npk = len(fir) // 12
    fir = fir[: npk * 12].reshape(npk, 12, 32)
    pk = np.zeros((npk, 1206), np.uint8)
    blk = pk[:, :1200].reshape(npk, 12, 100)
    blk[:, :, 0:2] = np.frombuffer(np.uint16(0xEEFF).tobytes(), np.uint8)
    rot = np.round(fir[:, :, 0]["azimuth"] * 100).astype(np.uint16)
    blk[:, :, 2:4] = rot.view(np.uint8).reshape(npk, 12, 2)
    ret = blk[:, :, 4:100].reshape(npk, 12, 32, 3)
    ret[:, :, :, 0:2] = fir["distance"].astype(np.uint16).view(np.uint8).reshape(npk, 12, 32, 2)
    ret[:, :, :, 2] = fir["intensity"]
    pk[:, 1205] = 0x21
    return pk, np.arange(npk, dtype=np.int64) * 553


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
    print(json.dumps({"stage": "preprocess", "sensor": ["HDL-64", "VLP-128", "HDL-32E"][sensor], "lasers": len(L),
                      "points": n, "wall_ms": round(el, 4), "device_ms": round(st[0] / reps, 4)}))
pk, ut = hdl32_packets(range(8))
dp = torch.from_numpy(pk.reshape(-1)).cuda()
du = torch.from_numpy(ut).cuda()
rec = torch.zeros(len(pk) * 384 * 32, dtype=torch.uint8, device="cuda")
for _ in range(3):
    ctx.velodyne_decode_device(dp.data_ptr(), du.data_ptr(), len(pk), rec.data_ptr())
ctx.set_timing(True)
ctx.stage_reset()
t0 = time.perf_counter()
for _ in range(reps):
    rs, rc = ctx.velodyne_decode_device(dp.data_ptr(), du.data_ptr(), len(pk), rec.data_ptr())
el = (time.perf_counter() - t0) / reps * 1e3
st = ctx.stage_times()["preprocess"]
dev_ms = st[0] / reps
nbytes = len(pk) * (1206 + 8 + 384 * 32)
print(json.dumps({"stage": "velodyne_decode", "packets": len(pk), "rotations": len(rc), "wall_ms": round(el, 4),
                  "device_ms": round(dev_ms, 4), "GBps": round(nbytes / (dev_ms * 1e-3) / 1e9, 1)}))
ctx.close()
