"""Host mirror of the FAST-LIO front-end hot path over the C-ABI.

Names follow the reference's interfaces so callers read like FAST-LIO
(upstream hku-mars src/laserMapping.cpp, include/ikd-Tree, IKFoM esekfom.hpp;
the Kodifly fork is an empty submodule in the reference, .gitmodules:1-3):

* :class:`IkdTreeGPU` — ``KD_TREE<PointType> ikdtree`` (``Build``, ``Add_Points``,
  ``Delete_Point_Boxes``, ``size``)
* :class:`LocalMap` — ``lasermap_fov_segment()``'s local-map cube
* :class:`HShareModelGPU` — ``h_share_model(state_ikfom&, dyn_share_datastruct&)``
  with its globals (``Nearest_Points``, ``point_selected_surf``, ``normvec``,
  ``feats_down_world``) exposed as getters
* :class:`EsekfGPU` — ``kf.update_iterated_dyn_share_modified(LASER_POINT_COV, solve_H_time)``

All compute runs in liblio_gpu.so on a gfx950 device; errors raise
:class:`lio_gpu._capi.LioError` (no CPU fallback).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import check, lib

_STATE_KEYS = ("pos", "rot", "offset_R_L_I", "offset_T_L_I", "vel", "bg", "ba", "grav")


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def default_match_params(**kw) -> _capi.MatchParams:
    """h_share_model constants [U]: gate sqdist[4] > 5, esti_plane 0.1f, s = 1 - 0.9|pd2|/sqrt(|p|) > 0.9."""
    p = _capi.MatchParams(5.0, 0.1, 0.9, 0.9)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def pose_from_arrays(R, t, R_LI=np.eye(3), t_LI=np.zeros(3), q=None, q_LI=None) -> _capi.Pose:
    """lio_pose; q / q_LI = the state's quaternions (w, x, y, z) — left zero (derived from R on the
    device side) when only matrices are given.  lio_pose is 32 doubles R, t, R_LI, t_LI, q, q_LI."""
    v = np.zeros(32, np.float64)
    v[0:9] = np.asarray(R, float).ravel()
    v[9:12] = np.asarray(t, float).ravel()
    v[12:21] = np.asarray(R_LI, float).ravel()
    v[21:24] = np.asarray(t_LI, float).ravel()
    if q is not None:
        v[24:28] = np.asarray(q, float).ravel()
    if q_LI is not None:
        v[28:32] = np.asarray(q_LI, float).ravel()
    return _capi.Pose.from_buffer_copy(v)


def pose_from_pose24(p24) -> _capi.Pose:
    """From a pose vector: R(9) t(3) R_LI(9) t_LI(3) [q(4) q_LI(4)] (synth.pose24 gives all 32)."""
    p24 = np.asarray(p24, float)
    if len(p24) >= 32:
        return pose_from_arrays(p24[0:9], p24[9:12], p24[12:21], p24[21:24], p24[24:28], p24[28:32])
    return pose_from_arrays(p24[0:9], p24[9:12], p24[12:21], p24[21:24])


def state_to_c(st: dict) -> _capi.State:
    s = _capi.State()
    for k in _STATE_KEYS:
        arr = getattr(s, k)
        for i, v in enumerate(np.asarray(st[k], float)):
            arr[i] = float(v)
    return s


def state_from_c(s: _capi.State) -> dict:
    return {k: np.array(list(getattr(s, k))) for k in _STATE_KEYS}


class IkdTreeGPU:
    """Dense-grid map in HBM standing in for the ikd-Tree (exact kNN)."""

    def __init__(self, cell_size: float = 1.0, downsample_size: float = 0.5, device: int = 0):
        self._h = C.c_void_p()
        self.device = device
        check(lib().lio_map_create(C.byref(_capi.MapParams(cell_size, downsample_size, device, 0)),
                                   C.byref(self._h)))

    def set_downsample_param(self, downsample_size: float):
        """``ikdtree.set_downsample_param(filter_size_map_min)``: in place, before Build."""
        check(lib().lio_map_set_params(self._h, C.byref(_capi.MapParams(0.0, downsample_size, self.device, 0))))

    def Build(self, points: np.ndarray):
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        check(lib().lio_map_build(self._h, _fp(pts), len(pts)))

    def Build_device(self, ptr: int, n: int):
        """Build from an xyz float32 buffer already in device memory (e.g. a torch tensor's data_ptr())."""
        check(lib().lio_map_build_device(self._h, C.c_void_p(ptr), n))

    def Build_pcd(self, path: str):
        """Build from the x y z columns of a saved PCD map."""
        check(lib().lio_map_build_pcd(self._h, path.encode()))

    def size(self) -> int:
        return int(lib().lio_map_size(self._h))

    def num_ids(self) -> int:
        """Ids ever inserted (alive + deleted); kNN ids index this space."""
        return int(lib().lio_map_num_ids(self._h))

    def by_id(self):
        """(xyz[num_ids,3], alive[num_ids]) for every id."""
        n = self.num_ids()
        xyz = np.empty((n, 3), np.float32)
        alive = np.empty(n, np.uint8)
        check(lib().lio_map_get_by_id(self._h, _fp(xyz), alive.ctypes.data_as(C.POINTER(C.c_uint8))))
        return xyz, alive.astype(bool)

    def Nearest_Search(self, points: np.ndarray, k_nearest: int = 5, max_dist: float = float("inf")):
        """ikdtree.Nearest_Search(point, k, Nearest_Points, Point_Distance, max_dist) [U] for a batch:
        (ids[n,k] into by_id (-1 where missing), sq-distances[n,k] (inf where missing))."""
        q = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        idx = np.empty((len(q), k_nearest), np.int32)
        d2 = np.empty((len(q), k_nearest), np.float32)
        check(lib().lio_map_nearest_search(self._h, _fp(q), len(q), k_nearest, max_dist,
                                           idx.ctypes.data_as(C.POINTER(C.c_int32)), _fp(d2)))
        return idx, d2

    def Add_Points(self, points: np.ndarray, downsample_on: bool) -> int:
        """ikdtree.Add_Points(PointToAdd, downsample_on) [U]; returns the reference's count."""
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        n = C.c_int64(0)
        check(lib().lio_map_add(self._h, _fp(pts), len(pts), 1 if downsample_on else 0, C.byref(n)))
        return int(n.value)

    def Add_Points_device(self, ptr: int, n: int, downsample_on: bool) -> int:
        out = C.c_int64(0)
        check(lib().lio_map_add_device(self._h, C.c_void_p(ptr), n, 1 if downsample_on else 0, C.byref(out)))
        return int(out.value)

    def Delete_Point_Boxes(self, boxes) -> int:
        """ikdtree.Delete_Point_Boxes(cub_needrm) [U]; boxes: (nb, 6) min xyz, max xyz."""
        b = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 6)
        n = C.c_int64(0)
        check(lib().lio_map_delete_boxes(self._h, _fp(b), len(b), C.byref(n)))
        return int(n.value)

    def points(self) -> np.ndarray:
        out = np.empty((self.size(), 3), np.float32)
        check(lib().lio_map_get_points(self._h, _fp(out)))
        return out

    def stats(self) -> dict:
        """Diagnostics (lio_map_get_stats): rebuilds so far, slot pool, sizes, last update's flags."""
        o = (C.c_int64 * 8)()
        check(lib().lio_map_get_stats(self._h, o))
        return dict(rebuilds=o[0], slots_cap=o[1], slots_used=o[2], alive=o[3], ids=o[4], cells=o[5], flags=o[6])

    def set_test_limits(self, slot_headroom: int = 0, dirty_cells: int = 0):
        """Test hook: a small slot pool / tombstone cell list, so the rebuild recovery paths run."""
        check(lib().lio_map_set_test_limits(self._h, int(slot_headroom), int(dirty_cells)))

    def grid(self):
        g = np.zeros(7)
        check(lib().lio_map_get_grid(self._h, _dp(g)))
        return dict(origin=g[0:3], cell=g[3], dims=g[4:7].astype(int))

    def close(self):
        # refused (and the handle kept) while an HShareModelGPU still uses this map
        if self._h and lib().lio_map_destroy(self._h) == 0:
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalMap:
    """``lasermap_fov_segment()`` [U]: the local-map cube around the LiDAR.

    ``update(pos_lid)`` returns the boxes to delete (``cub_needrm``), to be
    passed to :meth:`IkdTreeGPU.Delete_Point_Boxes`.  Defaults: cube_side_length
    1000 (kitti.launch:11), det_range 100 (kitti.yaml), MOV_THRESHOLD 1.5 [U].
    """

    def __init__(self, cube_len: float = 1000.0, det_range: float = 100.0, mov_threshold: float = 1.5):
        self.c = _capi.LocalMap()
        self.cube_len, self.det_range, self.mov_threshold = cube_len, det_range, mov_threshold

    def update(self, pos_lid) -> np.ndarray:
        pos = np.ascontiguousarray(pos_lid, dtype=np.float64).reshape(3)
        boxes = np.zeros((3, 6), np.float32)
        nb = C.c_int(0)
        check(lib().lio_localmap_update(C.byref(self.c), _dp(pos), self.cube_len, self.det_range,
                                        self.mov_threshold, _fp(boxes), C.byref(nb)))
        return boxes[: nb.value].copy()

    @property
    def box(self):
        return np.array(list(self.c.vertex_min)), np.array(list(self.c.vertex_max))


class HShareModelGPU:
    """``h_share_model`` on the GPU for one ``feats_down_body`` scan."""

    def __init__(self, tree: IkdTreeGPU, params: _capi.MatchParams | None = None):
        self.tree = tree
        self._h = C.c_void_p()
        self.params = params or default_match_params()
        check(lib().lio_ctx_create(tree._h, C.byref(self.params), C.byref(self._h)))
        self.n = 0

    def set_scan(self, body: np.ndarray):
        b = np.ascontiguousarray(body, dtype=np.float32).reshape(-1, 3)
        check(lib().lio_scan_set(self._h, _fp(b), len(b)))
        self.n = len(b)

    def set_scan_device(self, ptr: int, n: int):
        check(lib().lio_scan_set_device(self._h, C.c_void_p(ptr), n))
        self.n = n

    def bind_scan_device(self, ptr: int, n: int):
        """Use a caller-owned device scan in place (kept alive and unchanged by the caller)."""
        check(lib().lio_scan_bind_device(self._h, C.c_void_p(ptr), n))
        self.n = n

    def __call__(self, pose, converge: bool = True) -> np.ndarray:
        """One evaluation; ``pose`` is a lio Pose or a pose24 array. Returns sums[32]."""
        if not isinstance(pose, _capi.Pose):
            pose = pose_from_pose24(pose)
        sums = np.zeros(_capi.LIO_SUMS_LEN)
        check(lib().lio_match(self._h, C.byref(pose), 1 if converge else 0, _dp(sums)))
        return sums

    # ---- globals of the reference's h_share_model, for inspection / parity
    def nearest_points(self):
        idx = np.empty((self.n, 5), np.int32)
        d2 = np.empty((self.n, 5), np.float32)
        check(lib().lio_get_knn(self._h, idx.ctypes.data_as(C.POINTER(C.c_int32)), _fp(d2)))
        return idx, d2

    def normvec(self):
        abcd = np.empty((self.n, 4), np.float32)
        sel = np.empty(self.n, np.uint8)
        check(lib().lio_get_planes(self._h, _fp(abcd), sel.ctypes.data_as(C.POINTER(C.c_uint8))))
        return abcd, sel

    def world(self):
        w = np.empty((self.n, 3), np.float32)
        check(lib().lio_get_world(self._h, _fp(w)))
        return w

    def h_rows(self, max_rows: int):
        rows = np.empty((max(max_rows, 1), 7), np.float64)
        nr = C.c_int64(0)
        check(lib().lio_get_h_rows(self._h, _dp(rows), max_rows, C.byref(nr)))
        return rows[: min(nr.value, max_rows)], nr.value

    def knn_stats(self, pose):
        """Diagnostics: a kNN evaluation returning per-point (cells, points, last shell)."""
        if not isinstance(pose, _capi.Pose):
            pose = pose_from_pose24(pose)
        sums = np.zeros(_capi.LIO_SUMS_LEN)
        st = np.zeros((self.n, 3), np.int32)
        check(lib().lio_ctx_knn_stats(self._h, C.byref(pose), _dp(sums), st.ctypes.data_as(C.POINTER(C.c_int32))))
        return sums, st

    def preprocess_scan(self, raw: np.ndarray, imu_poses, end_pose, point_filter_num=4, blind=2.0,
                        filter_size_surf=0.5, time_field=4) -> int:
        """Raw scan -> Preprocess + UndistortPcl + downSizeFilterSurf straight into this scan
        (feats_down_body) on the device; returns feats_down_size."""
        from .filters import imu_poses_to_c

        raw = np.ascontiguousarray(raw, dtype=np.float32)
        prm = _capi.ScanPrepParams(point_filter_num, blind, filter_size_surf, time_field)
        n = C.c_int64(0)
        check(lib().lio_scan_preprocess(self._h, _fp(raw), len(raw), raw.shape[1], C.byref(prm),
                                        imu_poses_to_c(imu_poses), len(imu_poses), C.byref(end_pose), C.byref(n)))
        self.n = int(n.value)
        return self.n

    def undistorted(self) -> np.ndarray:
        """feats_undistort of the last preprocess_scan / preprocess_cloud2: the undistorted,
        time-sorted records (x, y, z, intensity, time, ...) before downSizeFilterSurf."""
        n = C.c_int64(0)
        stride = C.c_int(0)
        check(lib().lio_scan_get_undistorted(self._h, None, 0, C.byref(n), C.byref(stride)))
        out = np.empty((n.value, max(stride.value, 1)), np.float32)
        check(lib().lio_scan_get_undistorted(self._h, _fp(out), n.value, C.byref(n), C.byref(stride)))
        return out

    def keyframe_cloud(self, pose: _capi.Pose, T: np.ndarray) -> np.ndarray:
        """lio_scan_keyframe_cloud: (n, 4) float32 = T * pointBodyToWorld(pose, feats_undistort) with the
        intensity — fast_lio_sam's PosePcd cloud from /cloud_registered when T = pose_eig_.inverse()."""
        n = C.c_int64(0)
        T = np.ascontiguousarray(T, dtype=np.float64).reshape(16)
        check(lib().lio_scan_keyframe_cloud(self._h, C.byref(pose), _dp(T), None, 0, C.byref(n)))
        out = np.empty((n.value, 4), np.float32)
        check(lib().lio_scan_keyframe_cloud(self._h, C.byref(pose), _dp(T), _fp(out), n.value, C.byref(n)))
        return out

    def preprocess_cloud2(self, data, n_points: int, point_step: int, fields, imu_poses, end_pose, big_endian=False,
                          point_filter_num=4, blind=2.0, filter_size_surf=0.5) -> int:
        """preprocess_scan from sensor_msgs/PointCloud2 bytes; fields = 5 (offset, datatype[, scale]) for
        x, y, z, intensity, time (scaled to ms)."""
        from .filters import imu_poses_to_c
        from .formats import fields_to_c

        buf = np.frombuffer(bytes(data), np.uint8)
        prm = _capi.ScanPrepParams(point_filter_num, blind, filter_size_surf, 4)
        n = C.c_int64(0)
        check(lib().lio_scan_preprocess_cloud2(self._h, buf.ctypes.data_as(C.c_void_p), n_points, point_step,
                                               1 if big_endian else 0, fields_to_c(fields), C.byref(prm),
                                               imu_poses_to_c(imu_poses), len(imu_poses), C.byref(end_pose),
                                               C.byref(n)))
        self.n = int(n.value)
        return self.n

    def last_knn_pose24(self) -> np.ndarray:
        """pose24 of the last kNN evaluation (the pose Nearest_Points belong to)."""
        p = _capi.Pose()
        check(lib().lio_ctx_get_knn_pose(self._h, C.byref(p)))
        return np.concatenate([list(p.R), list(p.t), list(p.R_LI), list(p.t_LI), list(p.q),
                               list(p.q_LI)]).astype(np.float64)

    def map_incremental(self, pose, filter_size_map: float = 0.5) -> dict:
        """FAST-LIO ``map_incremental()`` [U]: add this scan to the map with the final pose.

        Uses Nearest_Points from the last kNN evaluation of this scan.
        """
        if not isinstance(pose, _capi.Pose):
            pose = pose_from_pose24(pose)
        st = _capi.IncrementalStats()
        check(lib().lio_map_incremental(self._h, C.byref(pose), float(filter_size_map), C.byref(st)))
        return {k: int(getattr(st, k)) for k, _ in _capi.IncrementalStats._fields_}

    def set_seed_scale(self, scale: float):
        """Test hook (lio_ctx_set_seed_scale): shrink the seeded kNN pass's bound by ``scale`` in
        (0, 1] so its not-full guard (whole-box far search) runs."""
        check(lib().lio_ctx_set_seed_scale(self._h, float(scale)))

    # ---- timing (HIP events on the context's stream)
    def set_timing(self, on: bool):
        check(lib().lio_ctx_set_timing(self._h, 1 if on else 0))

    def timing(self) -> dict:
        t = _capi.KernelTiming()
        check(lib().lio_ctx_get_timing(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in _capi.KernelTiming._fields_}

    def reset_timing(self):
        check(lib().lio_ctx_reset_timing(self._h))

    def close(self):
        if self._h:
            lib().lio_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EsekfGPU:
    """``esekfom::esekf::update_iterated_dyn_share_modified`` with the GPU h-model."""

    def __init__(self, model: HShareModelGPU, laser_point_cov: float = 0.001, max_iteration: int = 3,
                 epsi: float = 0.001):
        self.model = model
        self.params = _capi.IeskfParams(laser_point_cov, max_iteration, epsi)

    def update_iterated_dyn_share_modified(self, state: dict, P: np.ndarray):
        s = state_to_c(state)
        Pc = np.ascontiguousarray(P, dtype=np.float64).copy()
        st = _capi.IeskfStats()
        check(lib().lio_ieskf_update(self.model._h, C.byref(s), _dp(Pc), C.byref(self.params), C.byref(st)))
        stats = {k: getattr(st, k) for k, _ in _capi.IeskfStats._fields_}
        return state_from_c(s), Pc, stats

    def update_raw(self, s: _capi.State, P: np.ndarray, st: _capi.IeskfStats):
        """Same call on caller-owned ctypes state / float64 23x23 P / stats (updated in place):
        no per-call conversions (the shape a C++ caller of lio_ieskf_update has)."""
        check(lib().lio_ieskf_update(self.model._h, C.byref(s), P.ctypes.data_as(C.POINTER(C.c_double)),
                                     C.byref(self.params), C.byref(st)))
