"""CPU estimate of the ICP tile kernel's work for different source tilings.

The tile kernel's VALU work is ~ sum over tiles of the candidates in the tile's
box grown by the tile's largest NN distance (every one of the wave's 64 lanes
tests every candidate, active or not).  Exact NN by scipy cKDTree; candidates
counted from a 0.25 m target histogram.  Usage: icp_tiling_estimate.py A|B
"""
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, "fast-lio-sam_gps_amd")
from lio_gpu import synth  # noqa: E402

disp = (0.3, 1.5) if sys.argv[1] == "A" else (2.5, 4.0)
src, dst, T = synth.make_icp_pair(n_points=500_000, seed=4321, disp=disp)
d, _ = cKDTree(dst).query(src, k=1, workers=8)

h = 0.25
o = dst.min(0) - 10
ti = np.floor((dst - o) / h).astype(np.int64)
dims = ti.max(0) + 2
H = np.zeros(dims, np.int64)
np.add.at(H, (ti[:, 0], ti[:, 1], ti[:, 2]), 1)
S = np.pad(H.cumsum(0).cumsum(1).cumsum(2), ((1, 0), (1, 0), (1, 0)))


def boxcount(lo, hi):
    a = np.clip(np.floor((lo - o) / h).astype(np.int64), 0, dims - 1)
    b = np.clip(np.floor((hi - o) / h).astype(np.int64) + 1, 0, dims)
    return (S[b[0], b[1], b[2]] - S[a[0], b[1], b[2]] - S[b[0], a[1], b[2]] - S[b[0], b[1], a[2]]
            + S[a[0], a[1], b[2]] + S[a[0], b[1], a[2]] + S[b[0], a[1], a[2]] - S[a[0], a[1], a[2]])


def cost(tiles):
    tot = 0
    occ = 0
    for idx in tiles:
        p = src[idx]
        r = d[idx].max()
        tot += boxcount(p.min(0) - r, p.max(0) + r)
        occ += len(idx)
    nt = len(tiles)
    return f"tiles {nt:6d}  lanes {occ / nt / 64:.2f}  cand/tile {tot / nt:6.0f}  wave-cand {tot / 1e6:6.2f} M"


def cell_tiles(cell):
    c = np.floor((src - src.min(0)) / cell).astype(np.int64)
    key = (c[:, 2] * 100000 + c[:, 1]) * 100000 + c[:, 0]
    order = np.lexsort((np.arange(len(src)), key))
    ks = key[order]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    ends = np.r_[starts[1:], len(ks)]
    out = []
    for s, e in zip(starts, ends):
        n = e - s
        k = -(-n // 64)
        for t in range(k):
            out.append(order[s + n * t // k: s + n * (t + 1) // k])
    return out


def part1by2(v):
    v = v.astype(np.uint64) & np.uint64(0x1FFFFF)
    for sh, m in ((32, 0x1F00000000FFFF), (16, 0x1F0000FF0000FF), (8, 0x100F00F00F00F00F), (4, 0x10C30C30C30C30C3),
                  (2, 0x1249249249249249)):
        v = (v | (v << np.uint64(sh))) & np.uint64(m)
    return v


def morton(q):
    c = np.floor((src - src.min(0)) / q).astype(np.int64)
    return part1by2(c[:, 0]) | (part1by2(c[:, 1]) << np.uint64(1)) | (part1by2(c[:, 2]) << np.uint64(2))


def morton_chunks(q):
    order = np.argsort(morton(q), kind="stable")
    return [order[i:i + 64] for i in range(0, len(order), 64)]


def morton_blocks(q, level):
    """Morton blocks of 2^level fine cells per axis; consecutive blocks with a common parent merged
    while <= 64 points; blocks over 64 split into balanced Morton-contiguous chunks."""
    key = morton(q)
    order = np.argsort(key, kind="stable")
    ks = key[order] >> np.uint64(3 * level)
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    ends = np.r_[starts[1:], len(ks)]
    out = []
    cur_s = cur_e = None
    cur_parent = None
    for s, e in zip(starts, ends):
        n = e - s
        parent = int(ks[s]) >> 3
        if n > 64:
            if cur_s is not None:
                out.append(order[cur_s:cur_e])
                cur_s = None
            k = -(-n // 64)
            for t in range(k):
                out.append(order[s + n * t // k: s + n * (t + 1) // k])
            continue
        if cur_s is not None and parent == cur_parent and (e - cur_s) <= 64:
            cur_e = e
        else:
            if cur_s is not None:
                out.append(order[cur_s:cur_e])
            cur_s, cur_e, cur_parent = s, e, parent
    if cur_s is not None:
        out.append(order[cur_s:cur_e])
    return out


print("pair", sys.argv[1])
print("cells 2 m (current)        ", cost(cell_tiles(2.0)))
for q in (0.25, 0.5):
    print(f"morton chunks of 64, q={q}  ", cost(morton_chunks(q)))
for q, lv in ((0.5, 2), (0.25, 3), (0.5, 3)):
    print(f"morton blocks q={q} lv={lv}     ", cost(morton_blocks(q, lv)))
