"""Velodyne packet decode on the GPU (csrc/velodyne.hip) vs the oracle (oracle/oracle_velo.cpp):
records (all 32 bytes) and the pushed rotations bit-exact; and odometry_test's whole chain
(pcap -> HDL32ECapture -> Preprocessor -> LidarOdometry) through the compiled C++ API."""
import os
import subprocess

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc
from test_velodyne import packets_from_rotations, random_packets, write_pcap

pytestmark = pytest.mark.gpu
EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "b-shot-slam_amd", "bin",
                   "odometry_headless")


@pytest.fixture(scope="module")
def ctx():
    c = bshot_py.Context(0)
    yield c
    c.close()


def _rec_equal(a, b):
    """records equal field by field, float64 fields bit for bit (struct padding is indeterminate)"""
    assert len(a) == len(b)
    for f in ("azimuth", "vertical"):
        np.testing.assert_array_equal(a[f].view(np.uint64), b[f].view(np.uint64), err_msg=f)
    for f in ("distance", "intensity", "id", "time"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


def _check(ctx, pk, ut, maxl, sf):
    rec, rs, rc = ctx.velodyne_decode(pk, ut, maxl, sf)
    orec, orc_cnt = orc.velodyne_decode(pk, ut, maxl, sf)
    np.testing.assert_array_equal(rc, orc_cnt)
    np.testing.assert_array_equal(rs, np.concatenate([[0], np.cumsum(rc)[:-1]]) if len(rc) else rs)
    _rec_equal(rec, orec)
    return rec, rc


@pytest.mark.parametrize("maxl,sf", [(32, 0), (32, 1), (32, 3), (16, 0), (16, 2), (32, -1)])
def test_random_packets_exact(ctx, maxl, sf):
    pk, ut = random_packets(100 + maxl + sf, 300)
    _check(ctx, pk, ut, maxl, sf)


def test_synthetic_rotations_exact(ctx):
    pk, ut = packets_from_rotations([0, 1, 2, 3])
    rec, rc = _check(ctx, pk, ut, 32, 0)
    assert len(rc) == 3 and all(c == 32 * 2170 for c in rc)
    _check(ctx, pk, ut, 32, 2)


def test_foreign_sensor_type_fails_loudly(ctx):
    pk, ut = random_packets(3, 8, sensor_type=0x21)
    pk[5, 1205] = 0x10
    with pytest.raises(bshot_py.BshotError):
        ctx.velodyne_decode(pk, ut)


def test_device_path(ctx):
    import torch
    pk, ut = packets_from_rotations([0, 1, 2])
    dp = torch.from_numpy(pk.reshape(-1)).cuda()
    du = torch.from_numpy(ut).cuda()
    out = torch.zeros(len(pk) * 384 * 32, dtype=torch.uint8, device="cuda")
    rs, rc = ctx.velodyne_decode_device(dp.data_ptr(), du.data_ptr(), len(pk), out.data_ptr())
    orec, ocnt = orc.velodyne_decode(pk, ut)
    np.testing.assert_array_equal(rc, ocnt)
    recs = out.cpu().numpy().view(bshot_py.LASER_DTYPE)
    got = np.concatenate([recs[s:s + c] for s, c in zip(rs, rc)])
    _rec_equal(got, orec)


def test_pcap_capture_preprocess_odometry_chain(tmp_path):
    pk, ut = packets_from_rotations([0, 1, 2, 3])
    path = tmp_path / "hdl32.pcap"
    write_pcap(path, pk, [(1_600_000_000 + i // 100, (i * 553) % 1_000_000) for i in range(len(pk))])
    frames, k = 3, 600
    traj = tmp_path / "traj.txt"
    out = subprocess.run([EXE, str(frames), str(k), "2", "CV", "1", str(path), str(traj)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [ln.split() for ln in out.stdout.splitlines() if ln.startswith("frame ")]
    assert len(lines) == frames
    rpk, rut = bshot_py.pcap_load(path)
    rec, cnt = orc.velodyne_decode(rpk, rut, 32, 0)
    v = sorted(bshot_py.HDL32_VERTICAL)
    oo = orc.Odometry(orc.params(num_keypoints=k))
    starts = np.concatenate([[0], np.cumsum(cnt)])
    for f, ln in enumerate(lines):
        xyz, _ = orc.preprocess(rec[starts[f]:starts[f + 1]], v, -0.6, -1950.0)
        st = oo.process(xyz)
        assert int(ln[2]) == len(xyz) and int(ln[3]) == st.n_inliers, (f, ln[:4], st.n_inliers)
        pose = np.array([float.fromhex(x) for x in ln[4:20]], np.float32)
        assert np.array_equal(pose.view(np.uint32), np.array(st.pose, np.float32).view(np.uint32)), f
    # odometry_test's trajectory file: "x y z" of every pose (default 6-significant-digit output), then ""
    rows = traj.read_text().split("\n")
    assert rows[frames] == "" and len([r for r in rows if r]) == frames
    for f, ln in enumerate(lines):
        pose = np.array([float.fromhex(x) for x in ln[4:20]], np.float32).reshape(4, 4)
        got = np.array([float(v) for v in rows[f].split()])
        assert np.allclose(got, pose[:3, 3], rtol=1e-5, atol=1e-3), (f, got, pose[:3, 3])
