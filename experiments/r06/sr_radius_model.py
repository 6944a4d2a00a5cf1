"""Work model (CPU, synthetic HDL-64 sweep) for k_seg_ratio's candidate streaming: candidates and cell
lookups per query for the product's radius ladder vs. a continuous-radius start bounded by an earlier
query's exact 300th-NN distance: R_q <= R' + |q - q'|.

usage: python experiments/r06/sr_radius_model.py [nsample]
"""
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, "b-shot-slam_amd")
import bshot_py  # noqa: E402

r, K = 3000.0, 300
xyz = bshot_py.synth_sweep(0)[0].astype(np.float32)
ok = np.isfinite(xyz).all(1) & ~(xyz == 0).all(1)
xyz = xyz[ok].astype(np.float64)
n = len(xyz)
c0 = r / 16
# ladder key order (csrc/grid.hip k_ladder_keys): finest cells c0/2
ix = np.floor(xyz / (c0 / 2)).astype(np.int64)
x3 = (ix >> 4) + (1 << 16)
key = (x3[:, 0] << 46) | (x3[:, 1] << 29) | (x3[:, 2] << 12)
for m in (3, 2, 1):
    cb = (((ix[:, 0] >> m) & 1) << 2) | (((ix[:, 1] >> m) & 1) << 1) | ((ix[:, 2] >> m) & 1)
    key |= cb << (3 * m)
key |= ((ix[:, 0] & 1) << 2) | ((ix[:, 1] & 1) << 1) | (ix[:, 2] & 1)
order = np.argsort(key, kind="stable")
P = xyz[order]
tree = cKDTree(P)
nsample = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
rng = np.random.default_rng(1)
# runs of 16 consecutive cell-order queries
starts = rng.choice(n - 32, nsample // 16, replace=False)
qi = np.unique((starts[:, None] + np.arange(16)[None, :]).ravel())
dd, _ = tree.query(P, K, distance_upper_bound=r)
dK = dd[:, -1]  # inf when fewer than K within r
cnt_in = lambda q, R: len(tree.query_ball_point(q, R))  # noqa: E731

# per-level cell counts (levels: cells c0/2, c0, 2c0, 4c0, 8c0)
cells = [c0 / 2, c0, 2 * c0, 4 * c0, 8 * c0]
tabs = []
for c in cells:
    k = np.floor(P / c).astype(np.int64)
    u, cts = np.unique(k, axis=0, return_counts=True)
    tabs.append({tuple(a): b for a, b in zip(u.tolist(), cts.tolist())})


def stream(q, R, L):
    """(candidates, cube cells, probed cells) of one for_candidates pass at radius R on level L"""
    c = cells[L]
    lim = R + 0.05
    lo = np.floor((q - lim) / c).astype(int)
    hi = np.floor((q + lim) / c).astype(int)
    cand = 0
    probes = 0
    ncube = int(np.prod(hi - lo + 1))
    t = tabs[L]
    for a in range(lo[0], hi[0] + 1):
        dx = max(a * c - q[0], 0, q[0] - (a + 1) * c)
        for b in range(lo[1], hi[1] + 1):
            dy = max(b * c - q[1], 0, q[1] - (b + 1) * c)
            for e in range(lo[2], hi[2] + 1):
                dz = max(e * c - q[2], 0, q[2] - (e + 1) * c)
                if dx * dx + dy * dy + dz * dz <= lim * lim:
                    probes += 1
                    cand += t.get((a, b, e), 0)
    return cand, ncube, probes


fr = [1 / 16, 1 / (8 * 2 ** .5), 1 / 8, 1 / (4 * 2 ** .5), 1 / 4, 1 / (2 * 2 ** .5), 1 / 2, 1 / 2 ** .5, 1.0]
gi = [1, 1, 1, 2, 2, 3, 3, 4, 4]  # levels here: +1 (level 0 = the finest c0/2)


def ladder_start(q, pct=80):
    own = [tabs[L].get(tuple(np.floor(q / cells[L]).astype(int).tolist()), 0) for L in range(5)]
    kf = 3.14159265 * 100 / pct
    for s in range(8):
        rc = r * fr[s] / cells[gi[s]]
        if own[gi[s]] * kf * rc * rc >= K:
            return s
    return 8


def ladder(q):
    cand = probes = rounds = 0
    for s in range(ladder_start(q), 9):
        rs = r * fr[s]
        c, nc, pr = stream(q, rs, gi[s])
        rounds += (nc + 63) // 64
        probes += pr
        if c < K and s < 8:
            continue  # skipped unstreamed (cube < max_nn)
        cand += c
        if s == 8 or cnt_in(q, rs) >= K:
            return cand, probes, rounds, cnt_in(q, rs)
    return cand, probes, rounds, 0


def level_for(R, ratio_max):
    L = 4
    while L > 0 and R / cells[L - 1] <= ratio_max:
        L -= 1
    # coarsest level whose cell >= R / ratio_max ... i.e. the finest with R / cell <= ratio_max
    return L


def bounded(q, Rb, ratio_max):
    R = min(Rb * (1 + 1e-5) + 0.01, r)
    L = level_for(R, ratio_max) if R < r else 4
    c, nc, pr = stream(q, R, L)
    inb = cnt_in(q, R)
    extra = (0, 0, 0)
    if inb < K and R < r:
        extra = stream(q, r, 4)
        inb = cnt_in(q, r)
    return c + extra[0], pr + extra[2], (nc + 63) // 64 + (extra[1] + 63) // 64, inb


res = {"ladder": []}
strategies = {"prev_2.83": (1, 2.83), "prev_2": (1, 2.0), "seed8_2.83": (8, 2.83), "seed16_2.83": (16, 2.83),
              "seed8_2": (8, 2.0)}
for k in strategies:
    res[k] = []
qset = set(qi.tolist())
for j in qi:
    q = P[j]
    res["ladder"].append(ladder(q))
    for name, (S, rm) in strategies.items():
        if S == 1:
            jp = j - 1
        else:
            jp = j - j % S
        if jp == j or jp < 0 or not np.isfinite(dK[jp]):
            res[name].append(ladder(q))
            continue
        delta = float(np.linalg.norm(q - P[jp]))
        res[name].append(bounded(q, dK[jp] + delta, rm))
print(f"n={n} sampled queries={len(qi)}")
for name, v in res.items():
    a = np.array(v, float)
    print(f"{name:12s} cand/query {a[:, 0].mean():7.1f}  probes {a[:, 1].mean():6.1f}  lookup rounds {a[:, 2].mean():5.2f}"
          f"  in-ball {a[:, 3].mean():6.1f}  in-ball>640 {np.mean(a[:, 3] > 640):.3f}")
