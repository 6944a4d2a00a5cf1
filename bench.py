#!/usr/bin/env python3
"""bench.py -- sweeps/s of the B-SHOT odometry hot path on MI355X (BASELINE.json metric).

One "step" = one synthetic Velodyne-64 sweep (N ~= 130k points, float32 mm, already resident in
HBM) through extract (SR + top-K + ISS) + describe (normals + SHOT LRF + histogram + B-SHOT) +
match (map query + Hamming) + RANSAC + gate + ICP + map update, i.e. bshot_odom_process_device.
Workload = BASELINE config 2 sizes (130k-pt HDL-64 sweep, 2048 keypoints) run as a sequence so
every step also matches against the map (configs[2] semantics).

Multi-GPU: `bench.py --gpus N` starts N ranks itself (a torch.distributed.run child, launched before
anything touches the GPU; the driver's own `torch.distributed.run ... bench.py --gpus N` works the
same). One process per GPU, each running its own sequence (scene seed 42 + rank): frames shard with
no data-path collective ("scaling": "weak"); with N > 1 every sweep's map offer (K x 60 B) is also
all-gathered over RCCL and inserted into per-rank GPU replica maps (BASELINE config 4, the map
B-SHOT set broadcast; --no-map-bcast turns it off).

Prints ONE JSON line (rank 0). Roofline / cpu_baseline fields: DESIGN.md "Measurement".
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "b-shot-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bshot_py  # noqa: E402
from dist_map import exchange_map_delta  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
L2_PEAK_GBPS = 34500.0  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md "L2 (per XCD)")


def pmc_kernel(stage, path=None):
    """Counters of the stage's kernel from the newest committed PMC summary (profiles/rNN_pmc.json,
    scripts/pmc_summary.py): HBM bytes per launch (rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE,
    separate passes) and, where collected, the SQ / TCC / TCP derived metrics."""
    import glob
    import re
    # the default configuration's sets only (rNN<letters>_pmc.json, e.g. r05x, r05za; config sets carry
    # a suffix: r04c_c5), newest last
    files = [path] if path else sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))
                                       if re.fullmatch(r"r\d\d[a-z]*_pmc\.json", os.path.basename(f)))
    if not files:
        return None, None
    try:
        ks = json.load(open(files[-1]))["kernels"]
        # the product instantiation of a kernel templated on its diagnostic counters (k_seg_ratio<false>)
        k = ks.get(f"bsk::k_{stage}<false>") or ks.get(f"bsk::k_{stage}")
        return (k or None), os.path.relpath(files[-1], ROOT)
    except (OSError, ValueError, KeyError):
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 warm-up sweeps, >= 200 timed sweeps (the sequence's map grows meanwhile)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--keypoints", type=int, default=2048)
    ap.add_argument("--sensor", type=int, default=0, help="0 HDL-64 (130k), 1 VLP-128 style (256k), 2 HDL-32E (--from-lasers only)")
    ap.add_argument("--shot-radius", type=float, default=3000.0)
    ap.add_argument("--map-bcast", action="store_true",
                    help="per-sweep map exchange between ranks (C++ over RCCL, into GPU replicas); on by default for N > 1")
    ap.add_argument("--no-map-bcast", action="store_true", help="N > 1 without the map exchange")
    ap.add_argument("--sim-peers", type=int, default=0,
                    help="N = 1: run the RCCL map exchange on a 1-rank communicator and insert this rank's batch "
                         "into P more replicas per sweep (bshot_odom_exchange_sim): the insert work of a job of 1 + P ranks")
    ap.add_argument("--xchg-lazy", action="store_true",
                    help="replica policy xchg_index 0: log the gathered offers in HBM, index replicas on read "
                         "(default: every exchange indexed into the replicas inside the sweep, on the iss stream)")
    ap.add_argument("--map-bcast-py", action="store_true",
                    help="with --map-bcast: the Python all_gather of host records into host replicas instead")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-upload-leg", action="store_true",
                    help="skip the second timed leg whose sweeps start in pinned host memory (upload inside the region)")
    ap.add_argument("--metrics", default=None, help="per-sweep JSON lines of rank 0 (bshot_odom_set_metrics_file)")
    ap.add_argument("--cpu-frames", type=int, default=5)
    ap.add_argument("--pmc-file", default=None,
                    help="PMC summary (scripts/prof_summary.py) of this configuration; default: the newest profiles/r*_pmc.json")
    ap.add_argument("--profile-stages", action="store_true", help="print per-stage ms to stderr")
    ap.add_argument("--no-stage-timing", action="store_true", help="no per-stage HIP events in the timed region")
    ap.add_argument("--depth", type=int, default=2, help="lookahead depth (1: next sweep only, 2: two sweeps)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="process sweeps strictly one after another (no lookahead of the next sweep's SR/ISS)")
    ap.add_argument("--ladder-grids", type=int, default=None, help="tuning knob: 2 or 4 kNN ladder grids")
    ap.add_argument("--opt", action="append", default=[], help="tuning knob name=value (bshot_odom_set_option)")
    ap.add_argument("--map-sync", action="store_true",
                    help="wait for every GPU map insert and read the map size back per sweep (odometry_test never "
                         "reads it; default: the insert stays stream-ordered before the next sweep's map query)")
    ap.add_argument("--shard-frames", action="store_true",
                    help="N > 1: ONE sequence over the ranks (BASELINE config 3 scaled, strong scaling): ranks 1..N-1 "
                         "extract every (N-1)-th sweep (A0-A7 + ISS) and send its record to rank 0, which runs the "
                         "chain (matching, RANSAC, ICP, map) in sweep order")
    ap.add_argument("--from-lasers", action="store_true",
                    help="each sweep starts as HBM-resident laser returns and runs the GPU preprocessor "
                         "(SURVEY 8f row 3: range image, ground + occlusion removal) before the odometry")
    return ap.parse_args()


def spawn_ranks(a):
    """--gpus N > 1 outside a torch.distributed launcher: run N ranks as a child launcher process and
    return its exit code (this process never touches the GPU)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def run_shard(a, json_out, rank, world, local, dist, torch):
    """--shard-frames: one synthetic sequence (seed 42) over `world` ranks. Rank r >= 1 extracts the
    sweeps f with f mod (world - 1) == r - 1 (bshot_odom_extract_device, with its own lookahead over
    its sweeps) and sends each record (K x 60 B + ISS points) to rank 0 over a gloo group; rank 0 runs
    the chain half on the records in sweep order (bshot_odom_process_record). value = timed sweeps /
    the max over ranks of the time from the shared start barrier to each rank's last sweep."""
    dev = torch.device("cuda", local)
    g = dist.new_group(backend="gloo")
    W = world - 1
    params = bshot_py.default_params(num_keypoints=a.keypoints, shot_radius=a.shot_radius)
    nframes = a.warmup + a.steps
    odo = bshot_py.Odometry(device=local, params=params)
    odo.set_option("map_sync", 0)
    stats = []
    npts = 0
    if rank == 0:
        def recv(f):
            src = 1 + f % W
            ln = torch.zeros(1, dtype=torch.int64)
            dist.recv(ln, src, group=g, tag=f)
            buf = torch.empty(int(ln.item()), dtype=torch.float32)
            dist.recv(buf, src, group=g, tag=f)
            return buf.numpy()
        refused = 0

        def chain(f):
            nonlocal refused
            try:
                return odo.process_record(recv(f))
            except bshot_py.BshotError as e:
                # a sweep with fewer than K keypoints described over another context's stale normals
                # (bshot_abi.h, BSHOT_ESTALE): the owner extracts it itself, from the sequence's state
                if e.code != bshot_py.ESTALE:
                    raise
                refused += 1
                pc = torch.from_numpy(bshot_py.synth_sweep(f, sensor=a.sensor, seed=42)[0]).to(dev)
                return odo.process_device(pc.data_ptr(), int(pc.shape[0]))
        for f in range(a.warmup):
            chain(f)
        dist.barrier(group=g)
        t0 = time.perf_counter()
        for f in range(a.warmup, nframes):
            st = chain(f)
            stats.append(st)
            npts += st.n_points
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    else:
        mine = [f for f in range(nframes) if f % W == rank - 1]
        frames = {}
        for f in mine:
            pc, _ = bshot_py.synth_sweep(f, sensor=a.sensor, seed=42)
            frames[f] = torch.from_numpy(pc).to(dev)
        torch.cuda.synchronize(dev)
        pending = []

        def extract(i):
            f = mine[i]
            if i + 1 < len(mine):
                nx = frames[mine[i + 1]]
                odo.set_next_device(nx.data_ptr(), int(nx.shape[0]))
            rec = torch.from_numpy(odo.extract_device(frames[f].data_ptr(), int(frames[f].shape[0])))
            ln = torch.tensor([rec.numel()], dtype=torch.int64)
            pending.append((dist.isend(ln, 0, group=g, tag=f), dist.isend(rec, 0, group=g, tag=f), ln, rec))

        nw = sum(1 for f in mine if f < a.warmup)
        for i in range(nw):
            extract(i)
        dist.barrier(group=g)
        t0 = time.perf_counter()
        for i in range(nw, len(mine)):
            extract(i)
        for w1, w2, _, _ in pending:
            w1.wait()
            w2.wait()
        odo.drain()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
    el_max = float(t.item())
    if rank == 0:
        hm = np.mean([list(s.host_ms) for s in stats], axis=0)
        line = {
            "metric": "Velodyne-64 sweeps/sec (extract+match+ICP)",
            "value": round(a.steps / el_max, 3),
            "unit": "sweeps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el_max / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{['HDL-64', 'VLP-128', 'HDL-32E'][a.sensor]} synthetic sequence (one), "
                                   f"{int(npts / max(1, len(stats)))} pts/sweep, K={a.keypoints}, SHOT r={a.shot_radius:g} mm, "
                                   "full extract+describe+match+RANSAC+ICP+map per sweep",
                       "keypoints": a.keypoints, "parallelism": f"frame-sharded: extract x{W} ranks, chain on rank 0"},
            "host_ms_per_sweep": dict(zip(bshot_py.FrameStats.HOST_PHASES, np.round(hm, 3).tolist())),
            "records_refused": refused,
        }
        print(json.dumps(line), file=json_out, flush=True)
    odo.close()
    dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))
    # the JSON line is the only output on stdout: whatever the libraries print there (RCCL's
    # version banner at communicator init when NCCL_DEBUG is set, ...) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; the launcher's world size is used", file=sys.stderr)
    a.map_bcast = (a.map_bcast or world > 1) and not a.no_map_bcast
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        if 0 < ndev < world:
            # a rehearsal on fewer GPUs than ranks (ranks share devices): flow only, no scaling claim
            print(f"bench.py: {world} ranks on {ndev} GPU(s): ranks share devices", file=sys.stderr)
            local %= ndev
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import torch

    if a.shard_frames and world > 1:
        run_shard(a, json_out, rank, world, local, dist, torch)
        return
    dev = torch.device("cuda", local)
    params = bshot_py.default_params(num_keypoints=a.keypoints, shot_radius=a.shot_radius)
    # steady state at both edges of the timed region: the last warm-up sweep starts the first timed
    # sweep's lookahead, and the last timed sweep starts the lookahead of `extra` sweeps past the
    # region, which finishes inside it (bshot_odom_drain) -- the region holds exactly K sweeps' work
    extra = 0 if a.no_prefetch else max(1, min(2, a.depth))
    nframes = a.warmup + a.steps + extra
    nwork = a.warmup + a.steps
    seed = 42 + rank
    # synthetic sequence for this rank, uploaded to HBM before timing
    t0 = time.time()
    frames = []
    lasers = []
    pre_ctx = None
    vert = bshot_py.sensor_vertical_angles(a.sensor)
    for f in range(nframes):
        if a.from_lasers:
            L = bshot_py.synth_lasers(f, sensor=a.sensor, seed=seed)
            lasers.append((torch.from_numpy(L.view(np.uint8)).to(dev), len(L)))
            frames.append(torch.zeros((len(L), 3), dtype=torch.float32, device=dev))
        else:
            pc, _ = bshot_py.synth_sweep(f, sensor=a.sensor, seed=seed)
            frames.append(torch.from_numpy(pc).to(dev))
    if a.from_lasers:
        pre_ctx = bshot_py.Context(local)
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    npts = [int(x.shape[0]) for x in frames]
    pre_done = [False] * nframes

    def prep(j):
        # the preprocessor of sweep j (device lasers -> device points; syncs for the point count)
        if not a.from_lasers or j >= nframes or pre_done[j]:
            return
        npts[j] = pre_ctx.preprocess_device(lasers[j][0].data_ptr(), lasers[j][1], vert, frames[j].data_ptr(),
                                            lasers[j][1], lowpt_th=-1950.0)
        pre_done[j] = True

    odo = bshot_py.Odometry(device=local, params=params)
    try:
        odo.set_option("map_sync", 1 if a.map_sync else 0)
    except bshot_py.BshotError:  # an older library (A/B runs against a previous build)
        pass
    if a.ladder_grids is not None:
        odo.set_option("ladder_grids", a.ladder_grids)
    if a.metrics and rank == 0:
        odo.set_metrics_file(a.metrics)
    if a.xchg_lazy:
        odo.set_option("xchg_index", 0)
    for kv in a.opt:
        name, val = kv.split("=")
        odo.set_option(name, int(val))
    tot_pts = 0
    xchg = None
    if a.map_bcast and world > 1 and not a.map_bcast_py:
        # the RCCL id travels once over the process group; the per-sweep exchange is the library's
        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(bshot_py.Exchange.unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        ok = 1
        try:
            xchg = bshot_py.Exchange(bytes(uid.cpu().numpy().tobytes()), world, rank, local, a.keypoints)
        except bshot_py.BshotError as e:
            print(f"rank {rank}: RCCL exchange unavailable ({e}); map offers go over torch.distributed", file=sys.stderr)
            ok, xchg = 0, None
        # every rank takes the same transport (a rank whose communicator failed would otherwise leave
        # the others waiting in the all-gather)
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            if xchg is not None:
                xchg.close()
                xchg = None
            a.map_bcast_py = True
    elif a.sim_peers > 0 and world == 1:
        xchg = bshot_py.Exchange(bshot_py.Exchange.unique_id(), 1, 0, local, a.keypoints)

    def step(i):
        # sweeps are preprocessed when first needed (this one or a lookahead)
        for j in (i, i + 1, i + 2):
            prep(j)
        if not a.no_prefetch and i + 1 < nframes:
            odo.set_next_device(frames[i + 1].data_ptr(), npts[i + 1])
            # depth 2: the sweep after next gets its grids/SR/ISS queued beside the next describe
            if a.depth >= 2 and i + 2 < nframes:
                odo.set_next2_device(frames[i + 2].data_ptr(), npts[i + 2])
        st = odo.process_device(frames[i].data_ptr(), npts[i])
        if xchg is not None:
            # C++ / RCCL: the sweep's map offer all-gathered from HBM into the GPU replicas, no host sync
            if a.sim_peers > 0:
                odo.exchange_sim(xchg, a.sim_peers)
            else:
                odo.exchange(xchg)
        elif a.map_bcast and world > 1:
            for r, rec in exchange_map_delta(odo.map_delta(), dist, dev):
                odo.replica_insert(r, rec)
        return st

    wc_sweeps = [] if os.environ.get("BENCH_INTERVALS") else None
    if wc_sweeps is not None:
        import ctypes

    def timed(stepf):
        # barrier + device sync on both sides of exactly K sweeps; the lookahead started by the last
        # timed sweep finishes inside the region (drain)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t_0 = time.perf_counter()
        st_, mk_ = [], []
        for i in range(a.warmup, nwork):
            st_.append(stepf(i))
            mk_.append(time.perf_counter())
            if wc_sweeps is not None:  # diagnostics (BENCH_INTERVALS): the work counters after every sweep
                wc_ = (ctypes.c_int64 * 12)()
                bshot_py.lib().bshot_work_counters(ctypes.c_void_p(odo.context()), wc_, 12)
                wc_sweeps.append(list(wc_))
        return t_0, st_, mk_

    for i in range(a.warmup):
        step(i)
    # HIP events cost host time on every launch they bracket: in the default run only the stage of
    # the roofline kernel (SR) is timed; --profile-stages times them all
    odo.set_option("timing_mask", -1 if a.profile_stages else 1 << 1)
    odo.set_timing(not a.no_stage_timing)
    odo.stage_reset()
    if pre_ctx is not None:
        pre_ctx.set_timing(True)
        pre_ctx.stage_reset()
    t0, stats, marks = timed(step)
    tot_pts = int(sum(npts[a.warmup:nwork]))
    odo.drain()  # the lookahead started by the last timed sweep finishes inside the region
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    stages = odo.stage_times()
    odo.set_timing(False)
    if pre_ctx is not None:
        stages["preprocess"] = pre_ctx.stage_times()["preprocess"]
        pre_ctx.set_timing(False)
    el_max = el
    if dist is not None:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_max = float(t.item())
    sweeps = a.steps * world
    value = sweeps / el_max

    wc_main = None
    if os.environ.get("BENCH_INTERVALS"):
        import ctypes
        wc = (ctypes.c_int64 * 12)()
        bshot_py.lib().bshot_work_counters(ctypes.c_void_p(odo.context()), wc, 12)
        wc_main = list(wc)
    used_xchg = xchg is not None  # the RCCL exchange ran in the timed region (its replica policy goes in the line)
    if xchg is not None:
        xchg.close()
        xchg = None
    # one odometry per device at a time: a second context's four streams share the process's four
    # hardware queues with the first one's (GPU_MAX_HW_QUEUES), which measured 15-20 % slower
    odo.close()

    # ---- second leg (same sequence, fresh odometry, after the first one is closed): the sweeps start in pinned host memory and each
    # one's upload (a kernel copy on the queue stream, bshot_odom_upload) is issued two sweeps ahead,
    # inside the timed region -- SURVEY.md §8(d)'s "from cloud upload" (the reference's setSrcFrame
    # copy). Reported beside `value` (which keeps the sweeps HBM-resident), never as it.
    upload_leg = None
    if not (a.no_upload_leg or a.from_lasers or a.no_prefetch or a.depth < 2):
        host = [f_.cpu().pin_memory() for f_ in frames]
        dbuf = [torch.empty_like(f_) for f_ in frames]
        odo2 = bshot_py.Odometry(device=local, params=params)
        try:
            odo2.set_option("map_sync", 1 if a.map_sync else 0)
        except bshot_py.BshotError:
            pass
        if a.ladder_grids is not None:
            odo2.set_option("ladder_grids", a.ladder_grids)
        for kv in a.opt:
            name, val = kv.split("=")
            odo2.set_option(name, int(val))
        uploaded = [False] * nframes

        def up(j):
            if j < nframes and not uploaded[j]:
                odo2.upload(dbuf[j].data_ptr(), host[j].data_ptr(), npts[j])
                uploaded[j] = True

        def step2(i):
            if i + 1 < nframes:
                up(i + 1)
                odo2.set_next_device(dbuf[i + 1].data_ptr(), npts[i + 1])
                if i + 2 < nframes:
                    up(i + 2)
                    odo2.set_next2_device(dbuf[i + 2].data_ptr(), npts[i + 2])
            return odo2.process_device(dbuf[i].data_ptr(), npts[i])

        # sweeps 0 and 1 arrive before the run; every later one is uploaded as the sweep after next,
        # on the stream its lookahead then runs on
        up(0)
        up(1)
        torch.cuda.synchronize(dev)
        for i in range(a.warmup):
            step2(i)
        u0, _, _ = timed(step2)
        odo2.drain()
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        ue = time.perf_counter() - u0
        if dist is not None:
            t = torch.tensor([ue], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ue = float(t.item())
        odo2.close()
        upload_leg = {"value": round(a.steps * world / ue, 3), "unit": "sweeps/s",
                      "ms_per_step": round(ue / a.steps * 1e3, 3),
                      "bytes_per_sweep": int(12 * np.mean(npts[a.warmup:nwork])),
                      "path": "pinned host memory -> HBM by a kernel copy on the queue stream, issued two sweeps "
                              "ahead (bshot_odom_upload), inside the timed region"}
        del host, dbuf

    # ---- roofline of the dominant kernel: SURVEY.md §8(d) algorithmic bytes / event-timed launches
    ctx = bshot_py.Context(local, params)
    last = frames[-1]
    ctx.set_cloud_device(last.data_ptr(), npts[-1])
    P_sr = ctx.radius_pairs(params.seg_radius)
    kst = [int(x) for x in ctx.knn_stats()]  # SR work counters of the same sweep (separate launch)
    k_eff = float(np.mean([s.n_keypoints for s in stats]))
    m_eff = float(np.mean([s.n_target for s in stats]))
    icp_it = float(np.mean([s.icp_iters for s in stats]))
    corr = float(np.mean([s.n_mutual for s in stats]))
    n_eff = float(np.mean(npts[a.warmup:nwork]))
    ctx.close()
    # the dominant kernel among those with an algorithmic-bytes figure (k_seg_ratio in every
    # configuration measured so far, profiles/*_kernel_stats.csv)
    dom = max(((k, v) for k, v in stages.items() if k in ("seg_ratio", "match", "icp")), key=lambda kv: kv[1][0])
    per_launch_ms = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in stages.items()}
    # algorithmic bytes per launch (DESIGN.md "Measurement"): pair-gather convention
    alg = {
        "seg_ratio": 12.0 * P_sr + 8.0 * n_eff,
        "match": 88.0 * k_eff * m_eff,
        "icp": 12.0 * (k_eff + m_eff),
    }
    dname = dom[0]
    roof = None
    if dname in alg and per_launch_ms[dname] > 0:
        t_launch = per_launch_ms[dname] * 1e-3
        pmc, psrc = pmc_kernel(dname, a.pmc_file)
        traffic = round(pmc["hbm_read_bytes"] + pmc["hbm_write_bytes"]) if pmc and "hbm_read_bytes" in pmc else None
        roof = {"kernel": dname, "ms_per_launch": round(per_launch_ms[dname], 4), "traffic": traffic,
                "traffic_unit": "HBM bytes/launch (PMC)", "pmc_source": psrc}
        if dname == "seg_ratio":
            # the bytes the launch actually moves: the float4 candidates the radius ladder streams
            # (64 per chunk) + query read + ratio write. The per-sweep footprint (2 MB cloud + grids)
            # sits in L2, so those bytes are L2-served: the memory level this kernel touches is L2.
            g = 16.0 * 64.0 * kst[5] + 20.0 * n_eff
            ach = g / t_launch / 1e9
            roof.update({"bound": "l2", "achieved": round(ach, 1), "peak": L2_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / L2_PEAK_GBPS, 4), "bytes_per_launch": g,
                         "candidates_per_query": round(64.0 * kst[5] / max(1, kst[0]), 1)})
        else:
            ach = alg[dname] / t_launch / 1e9
            roof.update({"bound": "l2", "achieved": round(ach, 1), "peak": L2_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / L2_PEAK_GBPS, 4), "bytes_per_launch": alg[dname]})
        if traffic is not None:
            roof["hbm_achieved"] = round(traffic / t_launch / 1e9, 1)
            roof["hbm_frac"] = round(traffic / t_launch / 1e9 / HBM_PEAK_GBPS, 5)
        if pmc:
            # what limits the kernel, from the SQ/TCC counters of the committed PMC passes
            roof["limiter"] = {k: pmc[k] for k in ("limiter", "valu_issue_frac", "lds_busy_frac", "lds_bank_conflict_frac",
                                                    "waves_per_cu", "wave_wait_frac", "wave_issue_stall_frac",
                                                    "l2_hit_rate") if k in pmc}
        # SURVEY.md 8(d) pair-gather convention (every in-radius pair counted as read): informational
        # only -- the radius ladder never reads most of those pairs, so it is no roofline fraction
        roof["alg_pair_gather_bytes"] = alg[dname]
        roof["alg_pair_gather_GBps"] = round(alg[dname] / t_launch / 1e9, 1)

    # ---- CPU baseline: the oracle (CPU restatement of the reference algorithm), rank 0 only
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import oracle_ref
        # thread counts mirror the reference: SR, ISS, Hamming, RANSAC, ICP single-threaded;
        # normals and SHOT OpenMP with min(12, nproc) threads (include/bshot_bits.h:62,120)
        nthr = oracle_ref.set_threads(min(12, os.cpu_count() or 1))
        op = oracle_ref.params(num_keypoints=a.keypoints, shot_radius=a.shot_radius)
        od = oracle_ref.Odometry(op)
        nf = a.cpu_frames

        def cpu_frame(o, f):
            if a.from_lasers:
                # the oracle preprocessor (std::map restatement) runs inside the timed CPU sample too
                L = lasers[f][0].cpu().numpy().view(bshot_py.LASER_DTYPE)
                xyz, _ = oracle_ref.preprocess(L, vert, -0.6, -1950.0)
                o.process(xyz)
            else:
                o.process(frames[f].cpu().numpy())

        # sweep 0 (the initial self-match) untimed: the sample is steady-state sweeps 1..nf
        cpu_frame(od, 0)
        t1 = time.perf_counter()
        for f in range(1, nf + 1):
            cpu_frame(od, f)
        ct = time.perf_counter() - t1
        cpu = {"value": round(nf / ct, 4), "unit": "sweeps/s", "cores": nthr, "kind": "port",
               "sample": ("preprocessor + " if a.from_lasers else "") +
                         f"sweeps 1..{nf} (after the untimed initial sweep 0) of the same synthetic sequence (N~{int(n_eff)}, K={a.keypoints}), full "
                         f"path, oracle/ C++ restatement (PCL unavailable); {ct:.1f} s; SR/ISS/Hamming/RANSAC/ICP "
                         f"1 thread, normals/SHOT {nthr} OpenMP threads as in the reference",
               "cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count()}
        # BASELINE.md's second variant: every core this process may use for the OpenMP stages
        # (normals, SHOT); the restatement's other stages stay sequential as in the reference
        try:
            n_all = len(os.sched_getaffinity(0))
        except AttributeError:
            n_all = os.cpu_count() or 1
        n_all = min(n_all, int(os.environ.get("OMP_NUM_THREADS", n_all)) or n_all)
        if n_all > nthr and not a.from_lasers:
            oracle_ref.set_threads(n_all)
            od2 = oracle_ref.Odometry(op)
            cpu_frame(od2, 0)
            t1 = time.perf_counter()
            for f in range(1, nf + 1):
                cpu_frame(od2, f)
            ct2 = time.perf_counter() - t1
            cpu["all_cores"] = {"value": round(nf / ct2, 4), "cores": n_all}

    if rank == 0:
        if os.environ.get("BENCH_INTERVALS"):
            iv = np.diff([t0] + marks) * 1e3
            # per sweep (timed order): ICP iterations, targets, mutual matches, inliers, host phase ms
            per = [[s.icp_iters, s.n_target, s.n_mutual, s.n_inliers, s.n_keypoints] + [round(x, 3) for x in s.host_ms]
                   for s in stats]
            print(json.dumps({"sweep_intervals_ms": np.round(iv, 3).tolist(), "work": wc_main, "per_sweep": per,
                              "work_per_sweep": wc_sweeps,
                              # CLOCK_MONOTONIC ms, the clock of BSHOT_GROW_TRACE's lines
                              "t0_ms": round(t0 * 1e3, 3), "marks_ms": np.round(np.array(marks) * 1e3, 3).tolist()}),
                  file=sys.stderr)
        if a.profile_stages:
            print(json.dumps({k: [round(v[0], 3), v[1]] for k, v in stages.items()}), file=sys.stderr)
            hm = np.mean([list(s.host_ms) for s in stats], axis=0)
            print(json.dumps({"host_ms_per_sweep": dict(zip(bshot_py.FrameStats.HOST_PHASES, np.round(hm, 3).tolist()))}),
                  file=sys.stderr)
        line = {
            "metric": "Velodyne-64 sweeps/sec (extract+match+ICP)",
            "value": round(value, 3),
            "unit": "sweeps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el_max / a.steps * 1e3, 3),
            # median interval between consecutive sweep completions on rank 0 (host clock; with the
            # lookahead a sweep's extract/describe overlap the previous sweep's matching)
            "ms_per_step_median": round(float(np.median(np.diff([t0] + marks))) * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": ("laser returns -> GPU preprocessor -> " if a.from_lasers else "") +
                                   f"{['HDL-64', 'VLP-128', 'HDL-32E'][a.sensor]} synthetic sequence, "
                                   f"{int(n_eff)} pts/sweep, K={a.keypoints}, SHOT r={a.shot_radius:g} mm, "
                                   f"full extract+describe+match+RANSAC+ICP+map per sweep",
                       "keypoints": a.keypoints, "points_per_sweep": int(n_eff), "target_M": int(m_eff),
                       "map_size_readback": bool(a.map_sync),
                       "icp_iters": icp_it, "mutual_corr": round(corr, 1), "parallelism": f"sequence per rank x{world}" +
                       ((" + map exchange over torch.distributed" if a.map_bcast_py else " + RCCL map exchange")
                        if a.map_bcast else "") +
                       (f" + RCCL map exchange (1 rank) with {a.sim_peers} simulated peers' replica inserts"
                        if a.sim_peers > 0 else "") +
                       ((" (replicas logged in HBM, indexed on read)" if a.xchg_lazy else
                         " (replicas indexed every sweep, inside the timed region)")
                        if used_xchg else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "upload_inclusive": upload_leg,
            "stage_ms_per_sweep": {k: round(v[0] / a.steps, 4) for k, v in stages.items() if v[1]},
            # main-thread host wall time per phase (mean over the timed sweeps; a prefetched sweep's
            # extract/describe ran on the worker thread, so those phases are near zero here)
            "host_ms_per_sweep": dict(zip(bshot_py.FrameStats.HOST_PHASES,
                                          np.round(np.mean([list(s.host_ms) for s in stats], axis=0), 3).tolist())),
        }
        print(json.dumps(line), file=json_out, flush=True)
    if xchg is not None:
        xchg.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
