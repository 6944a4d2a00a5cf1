"""Throughput mode with fewer GPUs than ranks (BASELINE config 4): two sequences
share one GPU as two odometry contexts in one process (each with its own streams), and after every
frame each publishes its map delta and inserts the other's into a replica -- the exchange bench.py
--map-bcast runs over RCCL, with the all-gather replaced by a direct hand-over.

Checks: every sequence's poses are bit-identical to the same sequence run alone (contexts do not
interfere), and every replica holds as many keypoints as the map it mirrors, frame after frame."""
import numpy as np
import pytest

import bshot_py

pytestmark = pytest.mark.gpu

FRAMES = 3


def _solo(seed):
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=600))
    try:
        poses = []
        for f in range(FRAMES):
            xyz, _ = bshot_py.synth_sweep(f, seed=seed)
            st = od.process(xyz)
            poses.append(np.array(st.pose, np.float32).view(np.uint32).copy())
        return poses
    finally:
        od.close()


def test_two_sequences_one_gpu_map_exchange():
    seeds = (42, 43)
    ref = {s: _solo(s) for s in seeds}
    ods = [bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=600)) for _ in seeds]
    try:
        for f in range(FRAMES):
            deltas = []
            for r, (od, seed) in enumerate(zip(ods, seeds)):
                xyz, _ = bshot_py.synth_sweep(f, seed=seed)
                st = od.process(xyz)
                assert np.array_equal(np.array(st.pose, np.float32).view(np.uint32), ref[seed][f]), (seed, f)
                deltas.append((r, od.map_delta(), st.map_size))
            for r, od in enumerate(ods):
                for r2, rec, size in deltas:
                    if r2 != r:
                        od.replica_insert(r2, rec)
                        assert od.replica_size(r2) == size, (r, r2, f)
    finally:
        for od in ods:
            od.close()
