"""Map-delta exchange between ranks (BASELINE config 4).

Each rank runs its own sequence; after every frame it publishes the keypoints it inserted into
its map (K records of 15 x 4 B: xyz, seg ratio, 11 B-SHOT words) and every other rank applies
them to a replica of that rank's map with the same host Map code, so replicas stay identical to
the owner's map (same insertion order -> same unordered_map iteration order).

One all_gather of the counts plus one all_gather of the padded records per frame (<= 246 KB at
K=4096): on xGMI that is microseconds, so no bucketing is needed. Records travel as int32 so the
bit patterns of the descriptor words are moved, never reinterpreted as floats.
"""
import numpy as np
import torch


def exchange_map_delta(rec: np.ndarray, dist, device) -> list:
    """All-gather this rank's map delta; returns [(rank, records)] for every OTHER rank."""
    world = dist.get_world_size()
    me = dist.get_rank()
    rec = np.ascontiguousarray(rec, np.float32).reshape(-1, 15)
    t = torch.from_numpy(rec.view(np.int32)).to(device)
    k = torch.tensor([t.shape[0]], dtype=torch.int64, device=device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k)
    counts = [int(x.item()) for x in ks]
    kmax = max(counts)
    if kmax == 0:
        return [(r, np.zeros((0, 15), np.float32)) for r in range(world) if r != me]
    pad = torch.zeros((kmax, 15), dtype=torch.int32, device=device)
    pad[: t.shape[0]] = t
    bufs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    out = []
    for r in range(world):
        if r != me:
            out.append((r, bufs[r][: counts[r]].cpu().numpy().view(np.float32).copy()))
    return out
