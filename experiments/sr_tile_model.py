"""Work model for a cell-tiled SR (CPU estimate on the synthetic HDL-64 sweep): per-query ladder
candidate counts vs. tiles of T hierarchically-sorted queries sharing one LDS-staged superset."""
import sys, numpy as np
from scipy.spatial import cKDTree
sys.path.insert(0, "b-shot-slam_amd")
import bshot_py

r, K = 3000.0, 300
xyz = bshot_py.synth_sweep(0)[0].astype(np.float64)
ok = np.isfinite(xyz).all(1) & ~(xyz == 0).all(1)
xyz = xyz[ok]
n = len(xyz)
c0 = r / 16
fr = np.array([1/16, 1/(8*2**.5), 1/8, 1/(4*2**.5), 1/4, 1/(2*2**.5), 1/2, 1/2**.5, 1.0])
gi = np.array([0, 0, 0, 1, 1, 2, 2, 3, 3])
tree = cKDTree(xyz)
d, _ = tree.query(xyz, K)
dK = d[:, -1]
step = np.searchsorted(fr * r, dK, side="right")  # first step with rs > dK
step = np.minimum(step, 8)
print("n", n, "step hist", np.bincount(step, minlength=9))
ic = np.floor(xyz / c0).astype(np.int64)
key = []
x3 = (ic >> 3) + (1 << 15)
k = (x3[:, 0] << 41) | (x3[:, 1] << 25) | (x3[:, 2] << 9)
for L in (2, 1, 0):
    k |= ((((ic[:, 0] >> L) & 1) << 2) | (((ic[:, 1] >> L) & 1) << 1) | ((ic[:, 2] >> L) & 1)) << (3 * L)
order = np.argsort(k, kind="stable")
P = xyz[order]; S = step[order]

def linf_count(ctr, rad):
    return np.asarray(tree.query_ball_point(ctr, rad, p=np.inf, return_length=True))

# per-query: stream each step from (its start ~ deciding step - 1) to the deciding step
pq = 0
for s in range(9):
    m = S == s
    if not m.any(): continue
    for s2 in (s - 1, s):
        if s2 < 0: continue
        rs = fr[s2] * r; c = c0 * 2 ** gi[s2]
        pq += linf_count(P[m][::8], rs + c / 2).sum() * 8
print(f"per-query candidates/query ~{pq / n:.0f}")
for T in (32, 64, 128):
    work = stage = 0
    nt = (n + T - 1) // T
    for t in range(nt):
        q = P[t * T:(t + 1) * T]; s = S[t * T:(t + 1) * T]
        for s2 in range(max(0, s.min() - 1), s.max() + 1):
            act = s >= s2
            if not act.any(): continue
            rs = fr[s2] * r; c = c0 * 2 ** gi[s2]
            lo, hi = q[act].min(0), q[act].max(0)
            cnt = linf_count((lo + hi) / 2, (hi - lo).max() / 2 + rs + c / 2)
            work += cnt * act.sum(); stage += cnt
    print(f"T={T}: tile scan candidates/query ~{work / n:.0f}, staged/query ~{stage / n:.1f}")

# tiles = runs of one level-L cell (split into chunks of <= T): staged superset size per tile step
for L in (0, 1, 2):
    ck = k[order] >> (3 * L)
    brk = np.flatnonzero(np.diff(ck)) + 1
    starts = np.concatenate([[0], brk]); ends = np.concatenate([brk, [n]])
    for T in (64,):
        sizes = []; stage = 0; tiles = 0; work = 0
        for a, b in zip(starts, ends):
            for t0 in range(a, b, T):
                t1 = min(b, t0 + T); tiles += 1
                q = P[t0:t1]; s = S[t0:t1]
                for s2 in range(max(0, s.min() - 1), s.max() + 1):
                    act = s >= s2
                    rs = fr[s2] * r; c = c0 * 2 ** gi[s2]
                    lo, hi = q[act].min(0), q[act].max(0)
                    cnt = int(linf_count((lo + hi) / 2, (hi - lo).max() / 2 + rs + c / 2))
                    sizes.append(cnt); stage += cnt; work += cnt * int(act.sum())
        sizes = np.array(sizes)
        print(f"L={L} T={T}: tiles {tiles} (avg {n / tiles:.1f} q), staged/query {stage / n:.1f}, "
              f"superset p50 {np.percentile(sizes, 50):.0f} p90 {np.percentile(sizes, 90):.0f} "
              f"scan/query {work / n:.0f} p99 {np.percentile(sizes, 99):.0f} max {sizes.max()}, frac>2048 {np.mean(sizes > 2048):.3f} >4096 {np.mean(sizes > 4096):.3f}")
