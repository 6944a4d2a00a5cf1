"""The drop-in C++ API (include/bshot/, myslam::LidarOdometry) driven exactly like
test/odometry_test.cpp:173-194, as a compiled program linked against libbshot_amd.so:
per-frame poses must equal the oracle's restatement of the same loop bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

pytestmark = pytest.mark.gpu
EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "b-shot-slam_amd", "bin",
                   "odometry_headless")


@pytest.mark.parametrize("frames,k,sr", [(3, 600, "CV"), (2, 2048, "CVS")])
def test_cpp_odometry_loop_matches_oracle(frames, k, sr):
    out = subprocess.run([EXE, str(frames), str(k), "0", sr], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [ln.split() for ln in out.stdout.splitlines() if ln.startswith("frame ")]
    assert len(lines) == frames
    oo = orc.Odometry(orc.params(num_keypoints=k, sr_type={"CV": 0, "CVS": 1, "CVSN": 2}[sr]))
    for f, ln in enumerate(lines):
        xyz, _ = bshot_py.synth_sweep(f)
        st = oo.process(xyz)
        assert int(ln[2]) == len(xyz) and int(ln[3]) == st.n_inliers, (f, ln[:4], st.n_inliers)
        pose = np.array([float.fromhex(v) for v in ln[4:20]], np.float32)
        assert np.array_equal(pose.view(np.uint32), np.array(st.pose, np.float32).view(np.uint32)), f


def test_cpp_preprocessor_fed_loop_matches_oracle():
    """odometry_test's full loop: laser returns -> myslam::Preprocessor::run -> Frame -> odometry
    (test/odometry_test.cpp:111-194), HDL-32E synthetic rotations."""
    frames, k = 3, 600
    out = subprocess.run([EXE, str(frames), str(k), "2", "CV", "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [ln.split() for ln in out.stdout.splitlines() if ln.startswith("frame ")]
    assert len(lines) == frames
    oo = orc.Odometry(orc.params(num_keypoints=k))
    v = sorted(bshot_py.sensor_vertical_angles(2))
    for f, ln in enumerate(lines):
        xyz, _ = orc.preprocess(bshot_py.synth_lasers(f, sensor=2), v, -0.6, -1950.0)
        st = oo.process(xyz)
        assert int(ln[2]) == len(xyz) and int(ln[3]) == st.n_inliers, (f, ln[:4], st.n_inliers)
        pose = np.array([float.fromhex(v) for v in ln[4:20]], np.float32)
        assert np.array_equal(pose.view(np.uint32), np.array(st.pose, np.float32).view(np.uint32)), f
