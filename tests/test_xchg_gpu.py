"""BASELINE config 4 / SURVEY.md §8e: the per-sweep map exchange between sequences (one per rank).

* RCCL path (host/xchg.cpp): a one-rank communicator on the box's single GPU all-gathers the sweep's
  map offer from device buffers into a GPU replica of the rank's own map (include_self); the replica
  must hold exactly the map the odometry itself matches against -- same entries, same libstdc++
  block order -- and the same size.
* Cross-sequence targets (option xseq_targets, the replicas' consumer): the replica's entries join the
  matching targets between the own map's and the ref keypoints.
* Two ranks (two processes sharing the GPU, gloo as the transport of the host records): every rank
  ends with identical replicas of every sequence, and its own poses are bit-identical to a solo run
  (the exchange never perturbs a sequence unless xseq_targets asks for it)."""
import hashlib
import os
import socket

import numpy as np
import pytest

import bshot_py

pytestmark = pytest.mark.gpu

K = 800


def _frames(seed=42, n=6):
    return [bshot_py.synth_sweep(f, seed=seed)[0][::2].copy() for f in range(n)]


def _u(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def test_rccl_exchange_self_replica():
    uid = bshot_py.Exchange.unique_id()
    x = bshot_py.Exchange(uid, 1, 0, 0, K)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
    try:
        prev = None
        for f, xyz in enumerate(_frames()):
            rq = None
            if prev is not None:
                rq = od.gpu_replica_query(0, prev[0][:3, 3])
            st = od.process(xyz)
            if prev is not None:
                tx, tb = od.target()
                m = len(tx) - prev[1]  # map entries, then the ref keypoints
                assert m == len(rq[0]) and m > 0
                assert np.array_equal(_u(tx[:m]), _u(rq[0])) and np.array_equal(tb[:m], rq[1]), f
            od.exchange(x, include_self=True)
            assert od.gpu_replica_size(0) == st.map_size, f
            prev = (np.array(st.pose, np.float32).reshape(4, 4), st.n_keypoints)
    finally:
        od.close()
        x.close()


@pytest.mark.parametrize("index,peers", [(1, 3), (0, 3), (1, 10)])
def test_exchange_sim_peers_replicas(index, peers):
    # bshot_odom_exchange_sim (bench.py --sim-peers): every simulated peer's replica receives this
    # rank's batch, so each must equal the own map (entries, block order, size) sweep after sweep --
    # indexed at once (xchg_index 1: batched inserts of up to 8 replicas; 10 peers take two batches)
    # or from the log on read (0)
    uid = bshot_py.Exchange.unique_id()
    x = bshot_py.Exchange(uid, 1, 0, 0, K)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
    od.set_option("xchg_index", index)
    try:
        prev = None
        for f, xyz in enumerate(_frames(n=4)):
            rq = od.gpu_replica_query(peers, prev[0][:3, 3]) if prev is not None else None
            st = od.process(xyz)
            if rq is not None:  # the last peer's replica is the own map this sweep's matching read
                tx, tb = od.target()
                m = len(tx) - prev[1]
                assert m == len(rq[0]) and m > 0
                assert np.array_equal(_u(tx[:m]), _u(rq[0])) and np.array_equal(tb[:m], rq[1]), f
            od.exchange_sim(x, peers)
            pos = np.array(st.pose, np.float32).reshape(4, 4)[:3, 3]
            ref = od.gpu_replica_query(1, pos)
            for r in range(1, peers + 1):
                assert od.gpu_replica_size(r) == st.map_size, (f, r)
                got = od.gpu_replica_query(r, pos)
                assert np.array_equal(_u(got[0]), _u(ref[0])) and np.array_equal(got[1], ref[1]), (f, r)
            assert od.gpu_replica_size(0) == 0  # this rank's own replica is not fed (include_self off)
            prev = (np.array(st.pose, np.float32).reshape(4, 4), st.n_keypoints)
    finally:
        od.close()
        x.close()


def test_exchange_log_replayed_in_order(monkeypatch):
    """Replica policy xchg_index 0: the exchange logs every gathered offer in HBM and indexes the
    replicas only when one is read: nine sweeps' offers accumulate (a 200 KB log holds four: it is replayed into the replicas three
    times on the way), and the replica read before the last sweep must equal the own map the last
    sweep's matching reads (entries, libstdc++ block order, descriptors)."""
    monkeypatch.setenv("BSHOT_XCHG_LOG_KB", "200")
    uid = bshot_py.Exchange.unique_id()
    x = bshot_py.Exchange(uid, 1, 0, 0, K)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
    od.set_option("xchg_index", 0)  # the lazy replica policy
    try:
        frames = _frames(n=10)
        prev = None
        for f, xyz in enumerate(frames):
            rq = od.gpu_replica_query(0, prev[0][:3, 3]) if f == len(frames) - 1 else None
            st = od.process(xyz)
            if rq is not None:
                tx, tb = od.target()
                m = len(tx) - prev[1]
                assert m == len(rq[0]) and m > 0
                assert np.array_equal(_u(tx[:m]), _u(rq[0])) and np.array_equal(tb[:m], rq[1])
            else:
                od.exchange(x, include_self=True)
            prev = (np.array(st.pose, np.float32).reshape(4, 4), st.n_keypoints)
        assert od.gpu_replica_size(0) > 0
    finally:
        od.close()
        x.close()


def test_xseq_targets_append_replicas():
    uid = bshot_py.Exchange.unique_id()
    x = bshot_py.Exchange(uid, 1, 0, 0, K)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
    od.set_option("xseq_targets", 1)
    try:
        kref = 0
        for f, xyz in enumerate(_frames(n=4)):
            st = od.process(xyz)
            if f > 0:
                tx, tb = od.target()
                m = (len(tx) - kref) // 2
                assert m > 0 and 2 * m + kref == len(tx)
                # own map entries, then the replica's copy of them, then the ref keypoints
                assert np.array_equal(_u(tx[:m]), _u(tx[m:2 * m])) and np.array_equal(tb[:m], tb[m:2 * m]), f
            od.exchange(x, include_self=True)
            kref = st.n_keypoints
    finally:
        od.close()
        x.close()


def _rank(rank, world, port, q):
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        frames = _frames(seed=42 + rank, n=5)
        solo = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
        solo_poses = [_u(solo.process(x).pose).copy() for x in frames]
        solo.close()
        od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
        bad = []
        for f, xyz in enumerate(frames):
            st = od.process(xyz)
            if not np.array_equal(_u(st.pose), solo_poses[f]):
                bad.append(f"pose {f}")
            deltas = [None] * world
            dist.all_gather_object(deltas, od.map_delta())
            for r in range(world):
                od.gpu_replica_insert(r, deltas[r])
            sizes = [None] * world
            dist.all_gather_object(sizes, st.map_size)
            got = [od.gpu_replica_size(r) for r in range(world)]
            if got != sizes:
                bad.append(f"sizes {f}: {got} vs {sizes}")
            digest = []
            for r in range(world):
                xyz_r, bits_r = od.gpu_replica_query(r, np.array([0.0, 800.0 * f, 0.0], np.float32))
                digest.append(hashlib.sha1(_u(xyz_r).tobytes() + bits_r.tobytes()).hexdigest())
            digests = [None] * world
            dist.all_gather_object(digests, digest)
            if not all(d == digests[0] for d in digests):
                bad.append(f"digests {f}")
        od.close()
        dist.destroy_process_group()
        q.put((rank, True if not bad else "; ".join(bad)))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(300)
def test_two_ranks_identical_replicas_and_solo_poses():
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}, res


def _rccl_rank(rank, world, port, q):
    """One rank on its own GPU: the sequence's map offers go over RCCL (host/xchg.cpp) into every
    rank's GPU replicas, including its own (include_self)."""
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        uid = [bshot_py.Exchange.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)  # the RCCL id travels once over the process group
        frames = _frames(seed=42 + rank, n=5)
        solo = bshot_py.Odometry(rank, bshot_py.default_params(num_keypoints=K))
        solo_poses = [_u(solo.process(x).pose).copy() for x in frames]
        solo.close()
        x = bshot_py.Exchange(uid[0], world, rank, rank, K)
        od = bshot_py.Odometry(rank, bshot_py.default_params(num_keypoints=K))
        ok = True
        for f, xyz in enumerate(frames):
            st = od.process(xyz)
            ok &= np.array_equal(_u(st.pose), solo_poses[f])
            od.exchange(x, include_self=True)
            sizes = [None] * world
            dist.all_gather_object(sizes, st.map_size)
            ok &= all(od.gpu_replica_size(r) == sizes[r] for r in range(world))
            digest = []
            for r in range(world):
                xyz_r, bits_r = od.gpu_replica_query(r, np.array([0.0, 800.0 * f, 0.0], np.float32))
                digest.append(hashlib.sha1(_u(xyz_r).tobytes() + bits_r.tobytes()).hexdigest())
            digests = [None] * world
            dist.all_gather_object(digests, digest)
            ok &= all(d == digests[0] for d in digests)
        od.close()
        x.close()
        dist.destroy_process_group()
        q.put((rank, bool(ok)))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))


def _gpu_count():
    import torch

    return torch.cuda.device_count()  # counting does not initialise the GPU


@pytest.mark.timeout(300)
@pytest.mark.skipif(_gpu_count() < 2, reason="needs 2 GPUs: a rank per GPU with an RCCL communicator between them "
                                           "(the 1-GPU box runs the 1-rank RCCL test and the 2-rank gloo test)")
def test_two_ranks_rccl_two_gpus():
    """BASELINE config 4 on 2 GPUs over RCCL: every rank's poses equal its solo run's, and both ranks
    hold identical replicas of both sequences' maps (entries, order, sizes)."""
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rccl_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}, res
