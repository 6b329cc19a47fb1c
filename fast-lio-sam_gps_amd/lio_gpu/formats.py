"""Wire / disk formats at the hot path's boundary, over the C-ABI.

* ``sensor_msgs/PointCloud2`` data <-> float records (``pcl::fromROSMsg`` /
  ``pcl::toROSMsg`` field copies; /root/reference/fast_lio_sam/include/pose_pcd.hpp:37-39,
  utilities.hpp:120-127), decoded/encoded on the GPU
* binary PCD writer (``pcl::io::savePCDFileBinary``, fast_lio_sam.cpp:925-932; layout as
  post_process/merge_pcds.py:107-119) and an ascii/binary PCD reader
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import check, lib
from .filters import _Handle

# sensor_msgs/PointField datatypes
INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 = range(1, 9)
_NP = {INT8: np.int8, UINT8: np.uint8, INT16: np.int16, UINT16: np.uint16, INT32: np.int32, UINT32: np.uint32,
       FLOAT32: np.float32, FLOAT64: np.float64}
# pcl::toROSMsg(pcl::PointCloud<pcl::PointXYZI>): x 0, y 4, z 8, intensity 16, point_step 32
POINTXYZI = ([(0, FLOAT32), (4, FLOAT32), (8, FLOAT32), (16, FLOAT32)], 32)


def fields_to_c(fields):
    """fields: list of (offset, datatype[, scale]) -> ctypes array."""
    arr = (_capi.CloudField * len(fields))()
    for k, f in enumerate(fields):
        arr[k].offset = int(f[0])
        arr[k].datatype = int(f[1])
        arr[k].scale = float(f[2]) if len(f) > 2 else 1.0
    return arr


class CloudCodec(_Handle):
    def decode(self, data: bytes | np.ndarray, n_points: int, point_step: int, fields, big_endian=False) -> np.ndarray:
        buf = np.frombuffer(bytes(data) if not isinstance(data, np.ndarray) else data.tobytes(), np.uint8)
        out = np.empty((n_points, len(fields)), np.float32)
        check(lib().lio_cloud2_decode(self._h, buf.ctypes.data_as(C.c_void_p), n_points, point_step,
                                      1 if big_endian else 0, fields_to_c(fields), len(fields),
                                      out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def encode(self, rec: np.ndarray, fields=POINTXYZI[0], point_step=POINTXYZI[1]) -> bytes:
        rec = np.ascontiguousarray(rec, dtype=np.float32)
        out = np.empty(len(rec) * point_step, np.uint8)
        check(lib().lio_cloud2_encode(self._h, rec.ctypes.data_as(C.POINTER(C.c_float)), len(rec), rec.shape[1],
                                      fields_to_c(fields), len(fields), point_step, out.ctypes.data_as(C.c_void_p)))
        return out.tobytes()

    def read_pcd(self, path: str, want=("x", "y", "z", "intensity")) -> np.ndarray:
        n = C.c_int64(0)
        check(lib().lio_pcd_read(None, path.encode(), None, 0, None, 0, C.byref(n)))
        names = (C.c_char_p * len(want))(*[w.encode() for w in want])
        out = np.empty((max(n.value, 1), len(want)), np.float32)
        check(lib().lio_pcd_read(self._h, path.encode(), names, len(want), out.ctypes.data_as(C.POINTER(C.c_float)),
                                 n.value, C.byref(n)))
        return out[: n.value]


def pcd_points(path: str) -> int:
    n = C.c_int64(0)
    check(lib().lio_pcd_read(None, path.encode(), None, 0, None, 0, C.byref(n)))
    return int(n.value)


def write_pcd_binary(path: str, rec: np.ndarray, names=("x", "y", "z", "intensity")):
    rec = np.ascontiguousarray(rec, dtype=np.float32)
    arr = (C.c_char_p * len(names))(*[s.encode() for s in names])
    check(lib().lio_pcd_write_binary(path.encode(), rec.ctypes.data_as(C.POINTER(C.c_float)), len(rec), rec.shape[1],
                                     arr))
