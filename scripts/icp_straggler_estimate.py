import sys, numpy as np
sys.path.insert(0, "fast-lio-sam_gps_amd")
from scipy.spatial import cKDTree
from lio_gpu import synth
disp = (0.3, 1.5) if sys.argv[1] == "A" else (2.5, 4.0)
src, dst, T = synth.make_icp_pair(n_points=500_000, seed=4321, disp=disp)
d, _ = cKDTree(dst).query(src, k=1, workers=8)
print("pair", sys.argv[1], "NN dist pct 50/90/99/max", np.percentile(d, [50, 90, 99, 100]).round(2))
# tiles: 2 m cells, id order within cell, balanced <= 64
c = np.floor((src - src.min(0)) / 2.0).astype(np.int64)
key = (c[:, 2] * 10000 + c[:, 1]) * 10000 + c[:, 0]
order = np.lexsort((np.arange(len(src)), key))
ks = key[order]
starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
ends = np.r_[starts[1:], len(ks)]
# target histogram 0.25 m for box counts
h = 0.25
o = dst.min(0) - 10
ti = np.floor((dst - o) / h).astype(np.int64)
dims = ti.max(0) + 2
H = np.zeros(dims, np.int64)
np.add.at(H, (ti[:, 0], ti[:, 1], ti[:, 2]), 1)
S = H.cumsum(0).cumsum(1).cumsum(2)
S = np.pad(S, ((1, 0), (1, 0), (1, 0)))
def boxcount(lo, hi):
    a = np.clip(np.floor((lo - o) / h).astype(np.int64), 0, dims - 1)
    b = np.clip(np.floor((hi - o) / h).astype(np.int64) + 1, 0, dims)
    return (S[b[0], b[1], b[2]] - S[a[0], b[1], b[2]] - S[b[0], a[1], b[2]] - S[b[0], b[1], a[2]]
            + S[a[0], a[1], b[2]] + S[a[0], b[1], a[2]] + S[b[0], a[1], a[2]] - S[a[0], a[1], a[2]])
tot_max = tot_q = 0
nt = 0
strag = 0
for s, e in zip(starts, ends):
    n = e - s
    k = -(-n // 64)
    for t in range(k):
        idx = order[s + n * t // k: s + n * (t + 1) // k]
        p = src[idx]; dd = d[idx]
        lo, hi = p.min(0), p.max(0)
        rmax = dd.max()
        med = np.median(dd)
        thr = max(2 * med, 1.0)
        keep = dd <= thr
        rq = dd[keep].max()
        strag += (~keep).sum()
        tot_max += boxcount(lo - rmax, hi + rmax)
        tot_q += boxcount(lo - rq, hi + rq) if keep.any() else 0
        nt += 1
print(f"tiles {nt} q/tile {len(src)/nt:.1f} cand/tile (box, B=max) {tot_max/nt:.0f}  (B=non-straggler max) {tot_q/nt:.0f}  stragglers {strag} ({100*strag/len(src):.2f}%)")
