"""Point-cloud filters around the hot path, over the C-ABI.

* :class:`VoxelGrid` — ``pcl::VoxelGrid<PointT>`` (PCL 1.10 ``applyFilter``):
  FAST-LIO's ``downSizeFilterSurf`` and the loop closure's ``voxelizePcd``
  (/root/reference/fast_lio_sam/include/utilities.hpp:161-183)
* :func:`voxelize_submap` — one side of ``LoopClosure::setSrcAndDstCloud``
  (loop_closure.cpp:42-67): ``transformPcd`` (utilities.hpp:132-143) per
  keyframe, concatenation, ``voxelizePcd``
* :class:`ScanPreprocessor` — FAST-LIO ``Preprocess`` selection +
  ``ImuProcess::UndistortPcl`` + ``downSizeFilterSurf`` for one raw scan

Point records are float rows ``[x, y, z, attr...]`` (3..8 floats); PCL's
PointXYZI is ``stride = 4``, FAST-LIO's PointXYZINormal-with-time is
``[x, y, z, intensity, time_ms]`` (time = the reference's ``curvature``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import check, lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class _Handle:
    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        check(lib().lio_filter_create(device, C.byref(self._h)))

    def close(self):
        if self._h:
            lib().lio_filter_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class VoxelGrid(_Handle):
    """``pcl::VoxelGrid``: every field averaged per voxel, output in voxel-index order."""

    def __init__(self, leaf=0.5, device: int = 0):
        super().__init__(device)
        self.setLeafSize(*(np.broadcast_to(np.asarray(leaf, np.float32), 3)))

    def setLeafSize(self, lx, ly, lz):
        self.leaf = np.array([lx, ly, lz], np.float32)

    def filter(self, pts: np.ndarray) -> np.ndarray:
        pts = np.ascontiguousarray(pts, dtype=np.float32)
        pts2 = pts.reshape(len(pts), -1)
        stride = pts2.shape[1]
        out = np.empty_like(pts2)
        m = C.c_int64(0)
        check(lib().lio_voxel_grid(self._h, _fp(pts2), len(pts2), stride, _fp(self.leaf), _fp(out), C.byref(m)))
        return out[: m.value].copy()


def voxelize_submap(clouds, poses, voxel_res: float, handle: VoxelGrid | None = None) -> np.ndarray:
    """``voxelizePcd(sum_k transformPcd(clouds[k], poses[k]), voxel_res)``; poses are 4x4 double."""
    h = handle or VoxelGrid(voxel_res)
    clouds = [np.ascontiguousarray(c, dtype=np.float32) for c in clouds]
    stride = clouds[0].shape[1] if clouds else 4
    seg = np.zeros(len(clouds) + 1, np.int64)
    for k, c in enumerate(clouds):
        seg[k + 1] = seg[k] + len(c)
    pts = np.ascontiguousarray(np.concatenate(clouds) if clouds else np.zeros((0, stride), np.float32))
    T = np.ascontiguousarray(np.stack([np.asarray(p, np.float64).reshape(4, 4) for p in poses])
                             if poses else np.zeros((0, 4, 4)), dtype=np.float64)
    out = np.empty((max(len(pts), 1), stride), np.float32)
    m = C.c_int64(0)
    check(lib().lio_submap_voxelize(h._h, _fp(pts), seg.ctypes.data_as(C.POINTER(C.c_int64)), len(clouds), stride,
                                    T.ctypes.data_as(C.POINTER(C.c_double)), float(voxel_res), _fp(out), C.byref(m)))
    return out[: m.value].copy()


def imu_poses_to_c(poses):
    """poses: list of dicts offset_time, acc, gyr, vel, pos, rot (3x3)  ->  ctypes array (lio_imu_pose is 22
    doubles in this order; filled through numpy, not element by element)."""
    n = len(poses)
    P = np.zeros((max(n, 1), 22), np.float64)
    for i, p in enumerate(poses):  # row slices assigned directly (no per-field temporaries)
        r = P[i]
        r[0] = p["offset_time"]
        r[1:4] = p["acc"]
        r[4:7] = p["gyr"]
        r[7:10] = p["vel"]
        r[10:13] = p["pos"]
        r[13:22] = np.ravel(p["rot"])
    assert C.sizeof(_capi.ImuPose) == 22 * 8
    return (_capi.ImuPose * max(n, 1)).from_buffer(P)


class ScanPreprocessor(_Handle):
    """Preprocess (point_filter_num, blind) + UndistortPcl + downSizeFilterSurf, to host memory."""

    def __init__(self, point_filter_num=4, blind=2.0, filter_size_surf=0.5, time_field=4, device: int = 0):
        super().__init__(device)
        self.params = _capi.ScanPrepParams(point_filter_num, blind, filter_size_surf, time_field)

    def process(self, raw: np.ndarray, imu_poses, end_pose) -> np.ndarray:
        raw = np.ascontiguousarray(raw, dtype=np.float32)
        stride = raw.shape[1]
        out = np.empty_like(raw)
        m = C.c_int64(0)
        arr = imu_poses_to_c(imu_poses)
        check(lib().lio_preprocess(self._h, _fp(raw), len(raw), stride, C.byref(self.params), arr, len(imu_poses),
                                   C.byref(end_pose), _fp(out), C.byref(m)))
        return out[: m.value].copy()
