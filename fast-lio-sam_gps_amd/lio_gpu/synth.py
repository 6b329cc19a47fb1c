"""Synthetic scan/map generator for the BASELINE.json configurations.

The reference publishes no datasets or fixtures for this path,
so every parity test and bench line runs on these seeded, analytic scenes
(SURVEY.md §8d):

* "urban canyon": ground plane z=0, facades at y=±15 m (20 m tall) and
  axis-aligned boxes (1–10 m sides, 200 per 400 m of street), seed 1234;
* maps: points sampled uniformly (by area) on the visible surfaces with
  σ=0.01 m noise along the normal, interior samples rejected, exact duplicates
  removed — the ikd-Tree ``Build`` input of a static map;
* scans: ray-cast LiDAR patterns (Ouster-64 rings, Livox rosette, KITTI 64
  beam) from a ground-truth IMU pose through the FAST-LIO extrinsic
  (``kitti.yaml:23-26``: R_LI = I, t_LI = (0.81, -0.32, 0.8)), range ≤ 100 m
  (``kitti.yaml:21`` det_range), σ=0.02 m range noise, emitted in the order
  PCL's VoxelGrid (leaf 0.5 m, ``kitti.launch:9``) would emit them, i.e. the
  ``feats_down_body`` order that reaches ``h_share_model``;
* the initial filter state is T_gt ⊞ δ, δ=(0.10,-0.08,0.05 m; 0.5°,-0.4°,1.0°).

Everything here is host-side numpy input generation; nothing is timed.
"""
from __future__ import annotations

import concurrent.futures
import dataclasses
import math
import os

import numpy as np

T_LI = np.array([0.81, -0.32, 0.8])
R_LI = np.eye(3)
STREET_HALF_W = 15.0
FACADE_H = 20.0
DENSITY_STREET_LEN_PER_MPTS = 400.0  # metres of street per 1M map points (≈19 pts/m²)


# ----------------------------------------------------------------------------
# small SO(3) helpers (quaternion order w, x, y, z)
# ----------------------------------------------------------------------------
def rotvec_to_quat(v):
    v = np.asarray(v, dtype=np.float64)
    th = np.linalg.norm(v)
    if th < 1e-15:
        return np.array([1.0, 0.5 * v[0], 0.5 * v[1], 0.5 * v[2]])
    s = math.sin(0.5 * th) / th
    return np.array([math.cos(0.5 * th), s * v[0], s * v[1], s * v[2]])


def quat_mul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([
        aw * bw - ax * bx - ay * by - az * bz,
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by + ay * bw + az * bx - ax * bz,
        aw * bz + az * bw + ax * by - ay * bx,
    ])


def quat_to_mat(q):
    w, x, y, z = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([
        [1 - (tyy + tzz), txy - twz, txz + twy],
        [txy + twz, 1 - (txx + tzz), tyz - twx],
        [txz - twy, tyz + twx, 1 - (txx + tyy)],
    ])


def rotvec_to_mat(v):
    return quat_to_mat(rotvec_to_quat(v))


# ----------------------------------------------------------------------------
# scene
# ----------------------------------------------------------------------------
@dataclasses.dataclass
class Scene:
    length: float
    boxes: np.ndarray  # (B, 6) xmin ymin zmin xmax ymax zmax

    @property
    def x_range(self):
        return -0.5 * self.length, 0.5 * self.length


def make_scene(length: float = 400.0, seed: int = 1234) -> Scene:
    rng = np.random.default_rng(seed)
    nb = max(1, int(round(200 * length / 400.0)))
    size = rng.uniform(1.0, 10.0, size=(nb, 3))
    size[:, 1] = np.minimum(size[:, 1], 8.0)
    cx = rng.uniform(-0.5 * length + 6, 0.5 * length - 6, size=nb)
    # keep a drivable lane around y≈0: boxes sit along the kerbs
    side = rng.choice([-1.0, 1.0], size=nb)
    cy = side * rng.uniform(4.0 + 0.5 * size[:, 1], STREET_HALF_W - 0.5 * size[:, 1] + 1e-3)
    cy = np.clip(cy, -STREET_HALF_W + 0.5 * size[:, 1], STREET_HALF_W - 0.5 * size[:, 1])
    boxes = np.stack([cx - 0.5 * size[:, 0], cy - 0.5 * size[:, 1], np.zeros(nb),
                      cx + 0.5 * size[:, 0], cy + 0.5 * size[:, 1], size[:, 2]], axis=1)
    return Scene(length=length, boxes=boxes)


def _inside_any_box(p: np.ndarray, boxes: np.ndarray, margin: float = 1e-3) -> np.ndarray:
    """Mask of points strictly inside some box (x-sorted slab sweep)."""
    order = np.argsort(p[:, 0], kind="stable")
    xs = p[order, 0]
    inside = np.zeros(len(p), dtype=bool)
    for b in boxes:
        lo = np.searchsorted(xs, b[0] + margin, side="left")
        hi = np.searchsorted(xs, b[3] - margin, side="right")
        if hi <= lo:
            continue
        idx = order[lo:hi]
        q = p[idx]
        m = ((q[:, 1] > b[1] + margin) & (q[:, 1] < b[4] - margin) &
             (q[:, 2] > b[2] + margin) & (q[:, 2] < b[5] - margin))
        inside[idx[m]] = True
    return inside


def _faces(scene: Scene):
    """Planar rectangles: (origin, u, v, normal, area)."""
    x0, x1 = scene.x_range
    L = scene.length
    W = 2 * STREET_HALF_W
    faces = [
        (np.array([x0, -STREET_HALF_W, 0.0]), np.array([L, 0, 0.0]), np.array([0, W, 0.0]), np.array([0, 0, 1.0])),
        (np.array([x0, -STREET_HALF_W, 0.0]), np.array([L, 0, 0.0]), np.array([0, 0, FACADE_H]), np.array([0, 1.0, 0])),
        (np.array([x0, STREET_HALF_W, 0.0]), np.array([L, 0, 0.0]), np.array([0, 0, FACADE_H]), np.array([0, -1.0, 0])),
    ]
    for b in scene.boxes:
        sx, sy, sz = b[3] - b[0], b[4] - b[1], b[5] - b[2]
        faces += [
            (np.array([b[0], b[1], b[5]]), np.array([sx, 0, 0.0]), np.array([0, sy, 0.0]), np.array([0, 0, 1.0])),
            (np.array([b[0], b[1], b[2]]), np.array([sx, 0, 0.0]), np.array([0, 0, sz]), np.array([0, -1.0, 0])),
            (np.array([b[0], b[4], b[2]]), np.array([sx, 0, 0.0]), np.array([0, 0, sz]), np.array([0, 1.0, 0])),
            (np.array([b[0], b[1], b[2]]), np.array([0, sy, 0.0]), np.array([0, 0, sz]), np.array([-1.0, 0, 0])),
            (np.array([b[3], b[1], b[2]]), np.array([0, sy, 0.0]), np.array([0, 0, sz]), np.array([1.0, 0, 0])),
        ]
    out = []
    for o, u, v, n in faces:
        out.append((o, u, v, n, float(np.linalg.norm(u) * np.linalg.norm(v))))
    return out


_SURFACE_CACHE: dict = {}


def sample_surface(scene: Scene, n_points: int, seed: int = 1234, sigma: float = 0.01,
                   x_window=None) -> np.ndarray:
    """Area-uniform surface samples (float32, no interior points, no duplicates).  Deterministic, so
    the full-size maps are generated once per process (cached; a copy is returned)."""
    key = (scene.length, scene.boxes.tobytes(), n_points, seed, sigma, None if x_window is None else tuple(x_window))
    if key not in _SURFACE_CACHE:
        if len(_SURFACE_CACHE) >= 3:
            _SURFACE_CACHE.pop(next(iter(_SURFACE_CACHE)))
        _SURFACE_CACHE[key] = _sample_surface(scene, n_points, seed, sigma, x_window)
    return _SURFACE_CACHE[key].copy()


def _sample_surface(scene: Scene, n_points: int, seed: int, sigma: float, x_window) -> np.ndarray:
    rng = np.random.default_rng(seed + 7)
    faces = _faces(scene)
    if x_window is not None:  # drop faces entirely outside the window; the rest is rejection-sampled
        lo, hi = x_window
        faces = [f for f in faces if not (max(f[0][0], f[0][0] + f[1][0] + f[2][0]) < lo or
                                          min(f[0][0], f[0][0] + f[1][0] + f[2][0]) > hi)]
    areas = np.array([f[4] for f in faces])
    O = np.stack([f[0] for f in faces])
    U = np.stack([f[1] for f in faces])
    V = np.stack([f[2] for f in faces])
    N = np.stack([f[3] for f in faces])
    pts = []
    need = n_points
    while need > 0:
        m = int(need * 1.15) + 1024
        fid = rng.choice(len(faces), size=m, p=areas / areas.sum())
        uv = rng.random((m, 2))
        p = O[fid] + uv[:, :1] * U[fid] + uv[:, 1:] * V[fid] + rng.normal(0, sigma, (m, 1)) * N[fid]
        if x_window is not None:
            p = p[(p[:, 0] >= x_window[0]) & (p[:, 0] <= x_window[1])]
        p = p[~_inside_any_box(p, scene.boxes)]
        pts.append(p.astype(np.float32))
        need -= len(p)
    p = np.ascontiguousarray(np.concatenate(pts)[:n_points], dtype=np.float32)
    # exact duplicates removed, first occurrence kept (np.unique(p, axis=0) semantics; a stable
    # lexsort of the coordinate bits instead of the structured sort: 10 M points 21 s -> 3 s)
    b = p.view(np.uint32).reshape(-1, 3)
    k1 = (b[:, 0].astype(np.uint64) << np.uint64(32)) | b[:, 1].astype(np.uint64)
    order = np.lexsort((b[:, 2], k1))
    s1, s2 = k1[order], b[order, 2]
    dup = (s1[1:] == s1[:-1]) & (s2[1:] == s2[:-1])
    if dup.any():
        keep = np.ones(len(p), bool)
        keep[order[1:][dup]] = False
        p = p[keep]
    return np.ascontiguousarray(p, dtype=np.float32)


# ----------------------------------------------------------------------------
# ray casting
# ----------------------------------------------------------------------------
def _raycast(scene: Scene, origin: np.ndarray, dirs: np.ndarray, max_range: float = 100.0) -> np.ndarray:
    """Distance to the first hit along each unit ray (inf = miss)."""
    n = len(dirs)
    best = np.full(n, np.inf)
    x0, x1 = scene.x_range
    with np.errstate(divide="ignore", invalid="ignore"):
        # ground z = 0
        t = -origin[2] / dirs[:, 2]
        p = origin + t[:, None] * dirs
        ok = (t > 0) & (p[:, 0] >= x0) & (p[:, 0] <= x1) & (np.abs(p[:, 1]) <= STREET_HALF_W)
        best = np.where(ok & (t < best), t, best)
        for yw in (-STREET_HALF_W, STREET_HALF_W):
            t = (yw - origin[1]) / dirs[:, 1]
            p = origin + t[:, None] * dirs
            ok = (t > 0) & (p[:, 0] >= x0) & (p[:, 0] <= x1) & (p[:, 2] >= 0) & (p[:, 2] <= FACADE_H)
            best = np.where(ok & (t < best), t, best)
        inv = 1.0 / dirs
        B = scene.boxes
        # only boxes within range of the origin
        near = (B[:, 3] > origin[0] - max_range) & (B[:, 0] < origin[0] + max_range)
        B = B[near]
        def chunk(s):
            with np.errstate(divide="ignore", invalid="ignore"):
                iv = inv[s:s + 8192]
                t0 = (B[None, :, 0:3] - origin[None, None, :]) * iv[:, None, :]
                t1 = (B[None, :, 3:6] - origin[None, None, :]) * iv[:, None, :]
                tmin = np.nanmax(np.minimum(t0, t1), axis=2)
                tmax = np.nanmin(np.maximum(t0, t1), axis=2)
                hit = (tmax >= tmin) & (tmax > 0) & (tmin > 0)
                th = np.where(hit, tmin, np.inf).min(axis=1)
                best[s:s + 8192] = np.minimum(best[s:s + 8192], th)

        starts = list(range(0, n, 8192))
        if len(starts) > 2:  # numpy releases the GIL on these array ops: chunks in parallel threads
            with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
                list(ex.map(chunk, starts))
        else:
            for s in starts:
                chunk(s)
    best[best > max_range] = np.inf
    return best


def _sph(el, az):
    ce = np.cos(el)
    return np.stack([ce * np.cos(az), ce * np.sin(az), np.sin(el)], axis=1)


def scan_pattern(kind: str, n: int, rng) -> np.ndarray:
    """Unit ray directions in the LiDAR frame, scan order."""
    if kind == "ouster64":
        rings = 64
        cols = n // rings
        el = np.deg2rad(np.linspace(-16.6, 16.6, rings))
        az = np.linspace(0, 2 * np.pi, cols, endpoint=False)
        E, A = np.meshgrid(el, az, indexing="ij")
        return _sph(E.ravel(), A.ravel())[:n]
    if kind == "kitti64":
        rings = 64
        cols = int(math.ceil(n / rings))
        el = np.deg2rad(np.linspace(-24.8, 2.0, rings))
        az = np.linspace(0, 2 * np.pi, cols, endpoint=False)
        E, A = np.meshgrid(el, az, indexing="ij")
        return _sph(E.ravel(), A.ravel())[:n]
    if kind == "livox":
        # non-repetitive rosette, 70.4° circular FOV looking along +x
        t = np.arange(n) * 1e-4
        r = np.deg2rad(35.2) * np.abs(np.cos(7.3 * t * 1000.0))
        ph = 2 * np.pi * 0.618034 * np.arange(n) + 0.0137 * t
        az = r * np.cos(ph)
        el = r * np.sin(ph)
        return _sph(el, az)
    if kind == "random":
        el = np.deg2rad(rng.uniform(-20, 10, n))
        az = rng.uniform(0, 2 * np.pi, n)
        return _sph(el, az)
    raise ValueError(kind)


@dataclasses.dataclass
class Scan:
    body: np.ndarray        # (n, 3) float32, LiDAR frame, VoxelGrid order
    pos_gt: np.ndarray      # IMU position
    rot_gt: np.ndarray      # IMU quaternion (w,x,y,z)
    pos_init: np.ndarray
    rot_init: np.ndarray


def voxel_order(p: np.ndarray, leaf: float = 0.5) -> np.ndarray:
    """Permutation PCL VoxelGrid would emit points in (leaf index ascending)."""
    ijk = np.floor(p.astype(np.float64) / leaf).astype(np.int64)
    mn = ijk.min(axis=0)
    ijk -= mn
    dims = ijk.max(axis=0) + 1
    lin = ijk[:, 0] + ijk[:, 1] * dims[0] + ijk[:, 2] * dims[0] * dims[1]
    return np.argsort(lin, kind="stable")


def make_scan(scene: Scene, n: int, kind: str, pos_gt, yaw_gt: float = 0.0, seed: int = 99,
              delta=(0.10, -0.08, 0.05, 0.5, -0.4, 1.0), sensor_noise: float = 0.02) -> Scan:
    rng = np.random.default_rng(seed)
    rot_gt = rotvec_to_quat([0.0, 0.0, yaw_gt])
    Rg = quat_to_mat(rot_gt)
    pos_gt = np.asarray(pos_gt, dtype=np.float64)
    RL = Rg @ R_LI
    tL = Rg @ T_LI + pos_gt
    dirs_l = scan_pattern(kind, n, rng)
    dirs_w = dirs_l @ RL.T
    rng_ = _raycast(scene, tL, dirs_w)
    miss = ~np.isfinite(rng_)
    tries = 0
    while miss.any():
        k = int(miss.sum())
        el = np.deg2rad(rng.uniform(-16.0, -3.0, k))
        az = rng.uniform(0, 2 * np.pi, k)
        dl = _sph(el, az)
        dirs_l[miss] = dl
        dirs_w[miss] = dl @ RL.T
        rng_[miss] = _raycast(scene, tL, dirs_w[miss])
        miss = ~np.isfinite(rng_)
        tries += 1
        if tries > 50:
            raise RuntimeError("ray casting did not converge")
    rr = rng_ + rng.normal(0.0, sensor_noise, n)
    pw = tL + rr[:, None] * dirs_w
    pb = (pw - tL) @ RL  # R_L^T (p - t_L)
    pb = pb.astype(np.float32)
    pb = pb[voxel_order(pb, 0.5)]
    dpos = np.array(delta[:3])
    drot = np.deg2rad(np.array(delta[3:]))
    pos_init = pos_gt + dpos
    rot_init = quat_mul(rot_gt, rotvec_to_quat(drot))
    return Scan(body=np.ascontiguousarray(pb), pos_gt=pos_gt, rot_gt=rot_gt,
                pos_init=pos_init, rot_init=rot_init)


# ----------------------------------------------------------------------------
# filter state helpers (IKFoM state_ikfom layout, see include/lio_gpu.h)
# ----------------------------------------------------------------------------
def initial_state(pos, rot) -> dict:
    return dict(pos=np.asarray(pos, float), rot=np.asarray(rot, float),
                offset_R_L_I=np.array([1.0, 0, 0, 0]), offset_T_L_I=T_LI.copy(),
                vel=np.zeros(3), bg=np.zeros(3), ba=np.zeros(3), grav=np.array([0, 0, -9.809]))


def initial_cov() -> np.ndarray:
    d = np.full(23, 1e-4)
    d[0:3] = 1e-2
    d[3:6] = 1e-3
    return np.diag(d)


def pose24(state: dict) -> np.ndarray:
    """lio_pose as a vector: row-major R, t, R_LI, t_LI, then the state quaternions rot, offset_R_L_I
    (w, x, y, z) that the kernels rotate with (32 doubles; the name predates the quaternions)."""
    R = quat_to_mat(state["rot"])
    RLI = quat_to_mat(state["offset_R_L_I"])
    return np.concatenate([R.ravel(), state["pos"], RLI.ravel(), state["offset_T_L_I"],
                           state["rot"], state["offset_R_L_I"]]).astype(np.float64)


# ----------------------------------------------------------------------------
# BASELINE.json configurations
# ----------------------------------------------------------------------------
CONFIGS = {
    # name: (map points, street length, scan points, scan kind)
    "C1": (200_000, 400.0, 16_384, "ouster64"),
    "C2": (1_000_000, 400.0, 65_536, "ouster64"),
    "C3": (5_000_000, 2000.0, 131_072, "livox"),
    "C5": (10_000_000, 4000.0, 120_000, "kitti64"),
}


def make_config(name: str, n_scans: int = 1, map_points: int | None = None, scan_points: int | None = None,
                seed: int = 1234):
    mp, L, sp, kind = CONFIGS[name]
    mp = map_points or mp
    sp = scan_points or sp
    scene = make_scene(L, seed)
    mappts = sample_surface(scene, mp, seed)
    scans = []
    for k in range(n_scans):
        x = -0.15 * L + k * 3.7
        scans.append(make_scan(scene, sp, kind, pos_gt=[x, 0.6 * math.sin(0.7 * k), 0.0],
                               yaw_gt=0.05 * math.sin(0.3 * k), seed=99 + k))
    return scene, mappts, scans


def make_icp_pair(n_points: int = 500_000, seed: int = 4321, voxel: float = 0.3,
                  disp=(0.3, 1.5), length: float = 400.0):
    """Two overlapping voxelized submaps; dst = T_disp * scene."""
    rng = np.random.default_rng(seed)
    scene = make_scene(length, 1234)

    # street window long enough to hold n_points occupied 0.3 m voxels (~2.1k per metre)
    half = float(np.clip(0.5 * n_points / 1900.0 + 5.0, 10.0, 0.5 * length - 1.0))

    def submap(xc, s):
        # dense surface sample in the window, PCL-VoxelGrid-style centroids
        raw = sample_surface(scene, int(n_points * 3.2), seed=s, x_window=(xc - half, xc + half))
        ijk = np.floor(raw.astype(np.float64) / voxel).astype(np.int64)
        ijk -= ijk.min(axis=0)
        dims = ijk.max(axis=0) + 1
        lin = ijk[:, 0] + ijk[:, 1] * dims[0] + ijk[:, 2] * dims[0] * dims[1]
        u, inv = np.unique(lin, return_inverse=True)
        cnt = np.bincount(inv)
        cen = np.stack([np.bincount(inv, raw[:, d].astype(np.float64)) for d in range(3)], 1) / cnt[:, None]
        cen = cen.astype(np.float32)
        if len(cen) > n_points:
            keep = np.sort(rng.choice(len(cen), n_points, replace=False))
            cen = cen[keep]
        return np.ascontiguousarray(cen)

    # same 120 m stretch of street, independent surface samples / voxelizations
    src = submap(0.0, seed)
    tgt = submap(0.0, seed + 1)
    ang = np.deg2rad(disp[1])
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    tdir = rng.normal(size=3)
    tdir /= np.linalg.norm(tdir)
    R = rotvec_to_mat(axis * ang)
    t = tdir * disp[0]
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    dst = (tgt.astype(np.float64) @ R.T + t).astype(np.float32)
    return src, np.ascontiguousarray(dst), T


# ----------------------------------------------------------------------------
# Raw scans for the preprocessing path
# ----------------------------------------------------------------------------
def rotz(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def make_raw_scan(scene: Scene, n: int = 120_000, kind: str = "kitti64", seed: int = 7, speed: float = 8.0,
                  yaw_rate: float = 0.3, duration: float = 0.1, imu_hz: float = 100.0, origin=(0.0, 0.0, 0.0),
                  yaw0: float = 0.0):
    """A raw, motion-distorted LiDAR sweep with per-point time offsets and the IMU poses of that sweep.

    The IMU moves from `origin` (heading yaw0) at constant speed and yaw rate; the sweep is
    ray-cast at the end pose and every point is re-expressed in the LiDAR frame of its own
    firing time (time = azimuth fraction * duration), so FAST-LIO's UndistortPcl maps it back.
    Returns (raw, imu_poses, end24): raw rows (x, y, z, intensity, time_ms) in firing order;
    imu_poses as the IMUpose list (set_pose6d: offset_time, acc, gyr, vel, pos, rot); end24 =
    pose24 of the IMU state at the sweep end (lio_pose layout).
    """
    o = np.asarray(origin, dtype=np.float64)

    def traj(t):
        yaw = yaw0 + yaw_rate * t
        if abs(yaw_rate) > 1e-12:
            dx = speed / yaw_rate * (math.sin(yaw) - math.sin(yaw0))
            dy = speed / yaw_rate * (math.cos(yaw0) - math.cos(yaw))
        else:
            dx, dy = speed * t * math.cos(yaw0), speed * t * math.sin(yaw0)
        return rotz(yaw), o + np.array([dx, dy, 0.0]), yaw

    R_e, p_e, yaw_e = traj(duration)
    sc = make_scan(scene, n, kind, pos_gt=p_e, yaw_gt=yaw_e, seed=seed)
    rng = np.random.default_rng(seed)
    pe = sc.body.astype(np.float64)  # LiDAR frame at the sweep end
    az = np.arctan2(pe[:, 1], pe[:, 0])
    order = np.argsort(az, kind="stable")
    pe, az = pe[order], az[order]
    t_ms = ((az + np.pi) / (2 * np.pi) * duration * 1000.0).astype(np.float32)
    w = (pe @ R_LI.T + T_LI) @ R_e.T + p_e  # world points
    raw = np.empty((len(pe), 5), np.float32)
    for i0 in range(0, len(pe), 4096):  # re-express at each firing time
        sl = slice(i0, i0 + 4096)
        t = t_ms[sl].astype(np.float64) / 1000.0
        yaw = yaw0 + yaw_rate * t
        c, s_ = np.cos(yaw), np.sin(yaw)
        if abs(yaw_rate) > 1e-12:
            px = o[0] + speed / yaw_rate * (s_ - math.sin(yaw0))
            py = o[1] + speed / yaw_rate * (math.cos(yaw0) - c)
        else:
            px = o[0] + speed * t * math.cos(yaw0)
            py = o[1] + speed * t * math.sin(yaw0)
        d = w[sl] - np.stack([px, py, np.full_like(px, o[2])], axis=1)
        imu = np.stack([c * d[:, 0] + s_ * d[:, 1], -s_ * d[:, 0] + c * d[:, 1], d[:, 2]], axis=1)  # R_t^T d
        raw[sl, :3] = ((imu - T_LI) @ R_LI).astype(np.float32)
    raw[:, 3] = rng.uniform(0, 255, len(pe)).astype(np.float32)
    raw[:, 4] = t_ms
    poses = []
    k = int(round(duration * imu_hz))
    for j in range(k + 1):
        t = j / imu_hz
        R, p, yaw = traj(t)
        vel = speed * np.array([math.cos(yaw), math.sin(yaw), 0.0])
        acc = speed * yaw_rate * np.array([-math.sin(yaw), math.cos(yaw), 0.0])
        poses.append(dict(offset_time=t, acc=acc, gyr=np.array([0.0, 0.0, yaw_rate]), vel=vel, pos=p, rot=R))
    q_e = np.array([math.cos(0.5 * yaw_e), 0.0, 0.0, math.sin(0.5 * yaw_e)])  # state rot (yaw-only)
    end24 = np.concatenate([R_e.ravel(), p_e, R_LI.ravel(), T_LI, q_e, [1.0, 0.0, 0.0, 0.0]]).astype(np.float64)
    return raw, poses, end24


def make_loop_stream(scene: Scene, n_out: int = 4, n_points: int = 120_000, kind: str = "kitti64",
                     x0: float | None = None):
    """A C5-style stream with a loop: n_out raw sweeps driving out along +x, then n_out driving back
    along -x 40 s later past the same places (fast_lio_sam's loop_detection_timediff_threshold is
    30 s, config.yaml).  Returns [(raw, imu_poses, end24, initial_state, timestamp)]: the initial
    state is the sweep-end IMU pose off by (0.10, -0.08, 0.05) m and (0.5, -0.4, 1.0) deg, as the
    other configurations' scans."""
    delta = rotvec_to_quat(np.deg2rad([0.5, -0.4, 1.0]))
    if x0 is None:
        x0 = -0.15 * scene.length + 0.9
    plan = [(x0 + 3.7 * k, 0.4 * math.sin(0.5 * k), 0.04 * math.sin(0.2 * k), 0.1 * k) for k in range(n_out)]
    plan += [(x0 + 3.7 * (n_out - 1 - j) + 1.5, -0.3 + 0.2 * math.sin(0.7 * j), math.pi + 0.03 * math.sin(0.4 * j),
              40.0 + 0.1 * j) for j in range(n_out)]
    out = []
    for k, (ox, oy, yaw0, t) in enumerate(plan):
        raw, poses, end24 = make_raw_scan(scene, n_points, kind, seed=777 + k, origin=(ox, oy, 0.0), yaw0=yaw0)
        R_e = end24[0:9].reshape(3, 3)
        q_e = rotvec_to_quat([0.0, 0.0, float(np.arctan2(R_e[1, 0], R_e[0, 0]))])
        st0 = initial_state(end24[9:12] + np.array([0.10, -0.08, 0.05]), quat_mul(q_e, delta))
        out.append((raw, poses, end24, st0, t))
    return out
