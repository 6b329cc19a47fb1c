"""Incremental map maintenance, CPU side.

The C restatement (oracle/lio_oracle.cpp DynMap / map_incremental) is checked
against a second, deliberately naive pure-Python restatement written straight
from the upstream pseudo-code [U]:
  ikd-Tree KD_TREE::Add_Points(PointToAdd, downsample_on) / Delete_Point_Boxes
  FAST-LIO laserMapping.cpp map_incremental() and lasermap_fov_segment()
(small sizes: the Python loops are O(n * map)).  Parity with the real
reference is unpinned (its front end is an empty submodule, .gitmodules:1-3).
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

f32 = np.float32


def calc_dist(a, b):
    d = (a - b).astype(f32)
    return f32(f32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])


def same_point(a, b):
    return all(abs(f32(a[i] - b[i])) < f32(1e-6) for i in range(3))


class PyMap:
    """ids = insertion order, tombstones; survivors of a box keep their id,
    new survivors get ids in input order at the end of each Add_Points call."""

    def __init__(self, xyz):
        self.xyz = [np.asarray(p, f32) for p in xyz]
        self.alive = [True] * len(self.xyz)

    def add(self, pts, downsample, ds=f32(0.5)):
        pts = [np.asarray(p, f32) for p in pts]
        if not downsample:
            self.xyz += pts
            self.alive += [True] * len(pts)
            return len(pts)
        ds = f32(ds)
        pend = [False] * len(pts)
        counter = 0
        for i, q in enumerate(pts):
            vmin = np.array([f32(np.floor(f32(q[d] / ds)) * ds) for d in range(3)], f32)
            vmax = (vmin + ds).astype(f32)
            mid = np.array([f32(np.float64(vmin[d]) + np.float64(f32(vmax[d] - vmin[d])) / 2.0) for d in range(3)], f32)
            inbox = lambda a: all(vmin[d] <= a[d] < vmax[d] for d in range(3))  # noqa: E731
            st_map = [k for k in range(len(self.xyz)) if self.alive[k] and inbox(self.xyz[k])]
            st_new = [j for j in range(i) if pend[j] and inbox(pts[j])]
            md = calc_dist(q, mid)
            win, wmap, wnew = q, -1, i
            for k in st_map:
                t = calc_dist(self.xyz[k], mid)
                if t < md:
                    md, win, wmap, wnew = t, self.xyz[k], k, -1
            for j in st_new:
                t = calc_dist(pts[j], mid)
                if t < md:
                    md, win, wmap, wnew = t, pts[j], -1, j
            if len(st_map) + len(st_new) > 1 or same_point(q, win):
                for k in st_map:
                    if k != wmap:
                        self.alive[k] = False
                for j in st_new:
                    if j != wnew:
                        pend[j] = False
                if wnew == i:
                    pend[i] = True
                counter += 1
        for i, q in enumerate(pts):
            if pend[i]:
                self.xyz.append(q)
                self.alive.append(True)
        return counter

    def arrays(self):
        return np.array(self.xyz, f32).reshape(-1, 3), np.array(self.alive, bool)


def py_map_incremental(pm, body, pose_knn, pose, fs=0.5, ds=0.5):
    wk_all = O.body_to_world(pose_knn, body)
    w_all = O.body_to_world(pose, body)
    xyz, alive = pm.arrays()
    ids = np.nonzero(alive)[0]
    to_add, no_need, skipped = [], [], 0
    for i in range(len(body)):
        w, wk = w_all[i], wk_all[i]
        if len(ids) == 0:
            to_add.append(w)
            continue
        d2 = np.array([calc_dist(wk, xyz[k]) for k in ids], f32)
        order = np.lexsort((ids, d2))[:5]  # (d2, id) ascending, unbounded
        near = [xyz[ids[o]] for o in order]
        mid = np.array([f32(np.floor(np.float64(w[d]) / fs) * fs + 0.5 * fs) for d in range(3)], f32)
        dist = calc_dist(w, mid)
        if all(abs(f32(near[0][d] - mid[d])) > 0.5 * fs for d in range(3)):
            no_need.append(w)
            continue
        need = True
        for j in range(5):
            if len(near) < 5:
                break
            if calc_dist(near[j], mid) < dist:
                need = False
                break
        if need:
            to_add.append(w)
        else:
            skipped += 1
    c = pm.add(to_add, True, ds)
    pm.add(no_need, False, ds)
    return dict(n_to_add=len(to_add), n_no_downsample=len(no_need), n_skipped=skipped, n_added_downsample=c)


def _cloud(rng, n, lo=-3.0, hi=3.0):
    return rng.uniform(lo, hi, size=(n, 3)).astype(f32)


def test_add_points_downsample_matches_python():
    rng = np.random.default_rng(5)
    base = _cloud(rng, 400)
    om, pm = O.OracleDynMap(base), PyMap(base)
    for step in range(3):
        # clustered adds so voxels get several candidates (existing + new)
        new = np.concatenate([_cloud(rng, 60), base[rng.integers(0, len(base), 20)] + rng.normal(0, 0.05, (20, 3))])
        new = new.astype(f32)
        c1 = om.add(new, True, 0.5)
        c2 = pm.add(new, True, 0.5)
        assert c1 == c2
        x1, a1 = om.by_id()
        x2, a2 = pm.arrays()
        np.testing.assert_array_equal(x1, x2)
        np.testing.assert_array_equal(a1, a2)


def test_add_points_no_downsample_and_delete_boxes():
    rng = np.random.default_rng(6)
    base = _cloud(rng, 300)
    om = O.OracleDynMap(base)
    assert om.add(_cloud(rng, 50), False) == 50
    assert om.num_ids() == 350 and om.size() == 350
    boxes = np.array([[-3, -3, -3, 0, 0, 0], [1, 1, 1, 2, 2, 2]], f32)
    xyz, alive = om.by_id()
    inside = np.zeros(len(xyz), bool)
    for b in boxes:
        inside |= np.all((xyz >= b[:3]) & (xyz < b[3:]), axis=1)
    assert om.delete_boxes(boxes) == int(inside.sum())
    _, alive2 = om.by_id()
    np.testing.assert_array_equal(alive2, ~inside)
    # kNN skips tombstones
    q = _cloud(rng, 40)
    idx, _ = om.knn(q, 5, 1e30)
    assert np.all(alive2[idx[idx >= 0]])


def test_map_incremental_matches_python():
    rng = np.random.default_rng(7)
    base = _cloud(rng, 500, -4, 4)
    om, pm = O.OracleDynMap(base), PyMap(base)
    for step in range(2):
        body = _cloud(rng, 120, -4, 4)
        pose = np.zeros(24)
        pose[0:9] = np.eye(3).ravel()
        pose[9:12] = rng.normal(0, 0.3, 3)
        pose[12:21] = np.eye(3).ravel()
        pose[21:24] = [0.1, -0.05, 0.02]
        pk = pose.copy()
        pk[9:12] += rng.normal(0, 0.01, 3)  # kNN done at a slightly different iterate
        s1 = om.map_incremental(body, pk, pose)
        s2 = py_map_incremental(pm, body, pk, pose)
        assert s1 == s2
        x1, a1 = om.by_id()
        x2, a2 = pm.arrays()
        np.testing.assert_array_equal(x1, x2)
        np.testing.assert_array_equal(a1, a2)
    assert s1["n_no_downsample"] + s1["n_to_add"] + s1["n_skipped"] == 120


def py_fov_segment(lm, pos, cube_len=1000.0, det=f32(100.0), mov=f32(1.5)):
    """lasermap_fov_segment() [U] in numpy float32/float64 as laserMapping."""
    if lm.get("init") is None:
        lm["min"] = np.array([f32(p - cube_len / 2.0) for p in pos], f32)
        lm["max"] = np.array([f32(p + cube_len / 2.0) for p in pos], f32)
        lm["init"] = True
        return []
    dist = [[f32(abs(pos[i] - np.float64(lm["min"][i]))), f32(abs(pos[i] - np.float64(lm["max"][i])))] for i in range(3)]
    thr = f32(mov * det)
    if not any(dist[i][0] <= thr or dist[i][1] <= thr for i in range(3)):
        return []
    nmin, nmax = lm["min"].copy(), lm["max"].copy()
    mov_dist = f32(max((cube_len - 2.0 * np.float64(mov) * np.float64(det)) * 0.5 * 0.9, np.float64(f32(det * f32(mov - 1)))))
    boxes = []
    for i in range(3):
        bmin, bmax = lm["min"].copy(), lm["max"].copy()
        if dist[i][0] <= thr:
            nmax[i] = f32(nmax[i] - mov_dist)
            nmin[i] = f32(nmin[i] - mov_dist)
            bmin[i] = f32(lm["max"][i] - mov_dist)
            boxes.append(np.concatenate([bmin, bmax]))
        elif dist[i][1] <= thr:
            nmax[i] = f32(nmax[i] + mov_dist)
            nmin[i] = f32(nmin[i] + mov_dist)
            bmax[i] = f32(lm["min"][i] + mov_dist)
            boxes.append(np.concatenate([bmin, bmax]))
    lm["min"], lm["max"] = nmin, nmax
    return boxes


def test_localmap_update_matches_python():
    """lio_localmap_update is host code in liblio_gpu.so (no device needed)."""
    from lio_gpu import frontend as F

    lm = F.LocalMap(cube_len=1000.0, det_range=100.0, mov_threshold=1.5)
    ref = {}
    traj = [np.array([0.0, 0.0, 0.0]) + np.array([37.0, -11.0, 0.5]) * k for k in range(14)]
    n_moves = 0
    for pos in traj:
        got = lm.update(pos)
        exp = py_fov_segment(ref, pos)
        assert len(got) == len(exp)
        for g, e in zip(got, exp):
            np.testing.assert_array_equal(g, np.asarray(e, f32))
        n_moves += len(got) > 0
        bmin, bmax = lm.box
        np.testing.assert_array_equal(bmin.astype(f32), ref["min"])
        np.testing.assert_array_equal(bmax.astype(f32), ref["max"])
    assert n_moves >= 1
