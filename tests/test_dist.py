"""Multi-rank map-delta exchange (bench.py --map-bcast, BASELINE config 4) on CPU with gloo,
world_size 2: after every frame each rank's replica of its peer's map must be identical (same
keypoints, same descriptors, same iteration order) to the map the peer owns."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(rank, frame, k=200):
    rng = np.random.default_rng(1000 * rank + frame)
    rec = np.zeros((k, 15), np.float32)
    rec[:, :3] = rng.random((k, 3), dtype=np.float32) * 40000 - 20000 + np.float32(800 * frame)
    rec[:, 3] = rng.random(k, dtype=np.float32)
    rec[:, 4:] = rng.integers(0, 2 ** 32, (k, 11), dtype=np.uint64).astype(np.uint32).view(np.float32)
    rec[0, 4] = np.array([0x7FC00001], np.uint32).view(np.float32)[0]  # NaN payload must survive
    return rec


def _worker(rank, world, port, q):
    import bshot_py
    from dist_map import exchange_map_delta

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        own = bshot_py.KeypointMap()
        replicas = {r: bshot_py.KeypointMap() for r in range(world) if r != rank}
        for frame in range(4):
            rec = _records(rank, frame)
            for row in rec:
                own.add(row[:3], float(row[3]), row[4:].view(np.uint32))
            got = exchange_map_delta(rec, dist, "cpu")
            assert [r for r, _ in got] == [r for r in range(world) if r != rank]
            for r, peer in got:
                assert np.array_equal(peer.view(np.uint32), _records(r, frame).view(np.uint32))
                for row in peer:
                    replicas[r].add(row[:3], float(row[3]), row[4:].view(np.uint32))
        mine = own.query([0, 0, 0], 1e6)
        views = [None] * world
        dist.all_gather_object(views, {"own": mine, "rep": {r: m.query([0, 0, 0], 1e6) for r, m in replicas.items()}})
        for r in range(world):
            if r == rank:
                continue
            theirs = views[r]["rep"][rank]
            assert np.array_equal(theirs[0], mine[0]) and np.array_equal(theirs[1], mine[1])
        q.put((rank, "ok", own.size()))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_map_delta_exchange_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=170) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    assert all(s == "ok" for _, s, _ in res), res
    assert all(n > 0 for _, _, n in res)
