"""ctypes binding of the CPU oracle (oracle/lio_oracle.cpp).

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the CHECKER / timed CPU baseline — never by the
product package.  Parity against the real reference is unpinned (see the
oracle header and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liblio_oracle.so")

_lib = None


class MatchParams(C.Structure):
    _fields_ = [("knn_range_sq", C.c_float), ("plane_thr", C.c_float),
                ("s_coef", C.c_double), ("s_gate", C.c_double)]


class State(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("rot", C.c_double * 4), ("offset_R_L_I", C.c_double * 4),
                ("offset_T_L_I", C.c_double * 3), ("vel", C.c_double * 3), ("bg", C.c_double * 3),
                ("ba", C.c_double * 3), ("grav", C.c_double * 3)]


class IcpParams(C.Structure):
    _fields_ = [("max_corr_dist", C.c_double), ("trans_eps", C.c_double), ("fitness_eps", C.c_double),
                ("max_iter", C.c_int), ("rot_eps", C.c_double), ("score_threshold", C.c_double),
                ("umeyama_float", C.c_int)]


# pcl::umeyama float summation orders (lio_oracle.cpp UmeyamaOrder); the sentinels are the GPU's
# (include/lio_gpu.h): -1 = the opt-in double statistics (LIO_ICP_UMEYAMA_DOUBLE), 0 = the default order 2
ORACLE_DOUBLE_STATS = -1
DEFAULT_UMEYAMA_ORDER = 2
UMEYAMA_ORDERS = {1: "sequential means, sequential sigma", 2: "sequential means, Eigen GEMM sigma kc(32 KiB L1)",
                  3: "sequential means, Eigen GEMM sigma kc(48 KiB L1)", 4: "packet-4 means, sequential sigma",
                  5: "packet-4 means, Eigen GEMM sigma kc(32 KiB L1)"}


def default_match_params():
    return MatchParams(5.0, 0.1, 0.9, 0.9)


def default_icp_params():
    # loop_closure.cpp:7-10, fast_lio_sam.cpp:73 (1.5 * 35 m), config.yaml:16; PCL's float Umeyama in the
    # Eigen 3.3 GEMM order (loop_closure.h:42), the GPU default
    return IcpParams(52.5, 0.01, 0.01, 50, 0.0, 1.5, DEFAULT_UMEYAMA_ORDER)


def double_icp_params():
    """the opt-in double statistics (GPU: LoopClosure(umeyama_float=DOUBLE_STATS))"""
    p = default_icp_params()
    p.umeyama_float = ORACLE_DOUBLE_STATS
    return p


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def sincos(a):
    """the restatement's fixed sin / cos (UndistortPcl's SO3 Exp; lio_oracle.cpp sincos_fixed)"""
    a = np.ascontiguousarray(a, dtype=np.float64)
    s = np.empty_like(a)
    c = np.empty_like(a)
    lib().orc_sincos(_p(a, C.c_double), len(a), _p(s, C.c_double), _p(c, C.c_double))
    return s, c


def set_sincos_libm(on: bool) -> bool:
    """UndistortPcl's Exp through libm sin / cos (measurement switch); returns the previous setting"""
    return bool(lib().orc_set_sincos_libm(1 if on else 0))


def umeyama_float(src, tgt, order, stats=False):
    """pcl::umeyama(src, tgt, false) in float, correspondence pairs in order, summation order `order`;
    stats: also (src mean, tgt mean, sigma 3x3) as float32"""
    src = np.ascontiguousarray(src, dtype=np.float32)
    tgt = np.ascontiguousarray(tgt, dtype=np.float32)
    T = np.zeros(16, np.float32)
    st = np.zeros(15, np.float32)
    assert lib().orc_umeyama_float(_p(src, C.c_float), _p(tgt, C.c_float), len(src), int(order), _p(T, C.c_float),
                                   _p(st, C.c_float)) == 0
    if stats:
        return T.reshape(4, 4), st[0:3], st[3:6], st[6:15].reshape(3, 3)
    return T.reshape(4, 4)


def eigen_gemm_kc(k, l1):
    return int(lib().orc_eigen_gemm_kc(int(k), int(l1)))


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_sincos.argtypes = [C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_map_build.restype = C.c_void_p
        L.orc_map_build.argtypes = [C.POINTER(C.c_float), C.c_int64]
        L.orc_map_free.argtypes = [C.c_void_p]
        L.orc_map_knn.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int64, C.c_int, C.c_float,
                                  C.POINTER(C.c_int32), C.POINTER(C.c_float), C.c_int]
        L.orc_esti_plane.argtypes = [C.POINTER(C.c_float), C.c_float, C.POINTER(C.c_float)]
        L.orc_body_to_world.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_float), C.c_int64,
                                        C.POINTER(C.c_float)]
        L.orc_h_share_model.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int64, C.POINTER(C.c_double),
                                        C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_uint8),
                                        C.POINTER(C.c_float), C.POINTER(MatchParams), C.POINTER(C.c_double),
                                        C.c_int]
        L.orc_ieskf_update.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int64, C.POINTER(State),
                                       C.POINTER(C.c_double), C.POINTER(MatchParams), C.c_double, C.c_int,
                                       C.c_double, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                       C.POINTER(State)]
        L.orc_icp_align.argtypes = [C.POINTER(C.c_float), C.c_int64, C.POINTER(C.c_float), C.c_int64,
                                    C.POINTER(IcpParams), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                    C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_double),
                                    C.c_int, C.c_int]
        vp, i64 = C.c_void_p, C.c_int64
        L.orc_dmap_create.restype = vp
        L.orc_dmap_create.argtypes = [C.POINTER(C.c_float), i64]
        L.orc_dmap_free.argtypes = [vp]
        L.orc_dmap_num_ids.restype = i64
        L.orc_dmap_num_ids.argtypes = [vp]
        L.orc_dmap_alive_count.restype = i64
        L.orc_dmap_alive_count.argtypes = [vp]
        L.orc_dmap_get.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_uint8)]
        L.orc_dmap_add.restype = i64
        L.orc_dmap_add.argtypes = [vp, C.POINTER(C.c_float), i64, C.c_int, C.c_float]
        L.orc_dmap_delete_boxes.restype = i64
        L.orc_dmap_delete_boxes.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
        L.orc_dmap_knn.argtypes = [vp, C.POINTER(C.c_float), i64, C.c_int, C.c_float, C.POINTER(C.c_int32),
                                   C.POINTER(C.c_float)]
        L.orc_dmap_tree.restype = vp
        L.orc_dmap_tree.argtypes = [vp]
        L.orc_map_incremental.argtypes = [vp, C.POINTER(C.c_float), i64, C.POINTER(C.c_double),
                                          C.POINTER(C.c_double), C.c_double, C.c_float, C.POINTER(C.c_int64)]
        L.orc_voxel_grid.restype = i64
        L.orc_voxel_grid.argtypes = [C.POINTER(C.c_float), i64, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_submap_voxelize.restype = i64
        L.orc_submap_voxelize.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_int64), C.c_int, C.c_int,
                                          C.POINTER(C.c_double), C.c_float, C.POINTER(C.c_float)]
        L.orc_set_sincos_libm.argtypes = [C.c_int]
        L.orc_umeyama_float.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), i64, C.c_int,
                                        C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_eigen_gemm_kc.restype = i64
        L.orc_eigen_gemm_kc.argtypes = [i64, i64]
        L.orc_preprocess.restype = i64
        L.orc_preprocess.argtypes = [C.POINTER(C.c_float), i64, C.c_int, C.c_int, C.c_float, C.c_float, C.c_int,
                                     C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_float)]
        _lib = L
    return _lib


class OracleMap:
    """Static kd-tree with ikd-Tree Nearest_Search result semantics."""

    def __init__(self, xyz: np.ndarray):
        self.xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        self.h = lib().orc_map_build(_p(self.xyz, C.c_float), len(self.xyz))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_map_free(self.h)
            self.h = None

    def knn(self, q, k=5, range_sq=5.0, threads=8):
        q = np.ascontiguousarray(q, dtype=np.float32)
        idx = np.empty((len(q), k), np.int32)
        d2 = np.empty((len(q), k), np.float32)
        rc = lib().orc_map_knn(self.h, _p(q, C.c_float), len(q), k, C.c_float(range_sq), _p(idx, C.c_int32),
                               _p(d2, C.c_float), threads)
        assert rc == 0
        return idx, d2


def esti_plane(pts5x3, thr=0.1):
    p = np.ascontiguousarray(pts5x3, dtype=np.float32).reshape(15)
    out = np.empty(4, np.float32)
    ok = lib().orc_esti_plane(_p(p, C.c_float), C.c_float(thr), _p(out, C.c_float))
    return bool(ok), out


def _pose32(p):
    """Pose vector R t R_LI t_LI [q q_LI] -> the oracle's 32 doubles (zero quaternions = derive from R)."""
    p = np.asarray(p, dtype=np.float64).ravel()
    out = np.zeros(32, np.float64)
    out[: min(len(p), 32)] = p[:32]
    return out


def body_to_world(pose24, body):
    pose24 = _pose32(pose24)
    body = np.ascontiguousarray(body, dtype=np.float32)
    out = np.empty_like(body)
    lib().orc_body_to_world(_p(pose24, C.c_double), _p(body, C.c_float), len(body), _p(out, C.c_float))
    return out


def h_share_model(omap: OracleMap, body, pose24, redo_knn, nn_idx, sel, planes, mp=None, threads=8):
    """One h-evaluation; nn_idx/sel/planes are updated in place. Returns sums[32]."""
    mp = mp or default_match_params()
    body = np.ascontiguousarray(body, dtype=np.float32)
    pose24 = _pose32(pose24)
    sums = np.zeros(32, np.float64)
    rc = lib().orc_h_share_model(omap.h, _p(body, C.c_float), len(body), _p(pose24, C.c_double), int(redo_knn),
                                 _p(nn_idx, C.c_int32), _p(sel, C.c_uint8), _p(planes, C.c_float),
                                 C.byref(mp), _p(sums, C.c_double), threads)
    assert rc == 0
    return sums


def state_to_c(st: dict) -> State:
    s = State()
    for k in ("pos", "rot", "offset_R_L_I", "offset_T_L_I", "vel", "bg", "ba", "grav"):
        arr = getattr(s, k)
        for i, v in enumerate(st[k]):
            arr[i] = float(v)
    return s


def state_from_c(s: State) -> dict:
    return {k: np.array(list(getattr(s, k))) for k, _ in State._fields_}


def ieskf_update(omap: OracleMap, body, state: dict, P, mp=None, R=0.001, max_iter=3, limit=0.001, threads=8,
                 knn_state=False):
    """(state, P, stats, trace[, state of the last kNN evaluation when knn_state])"""
    mp = mp or default_match_params()
    body = np.ascontiguousarray(body, dtype=np.float32)
    s = state_to_c(state)
    sk = State()
    Pc = np.ascontiguousarray(P, dtype=np.float64).copy()
    stats = np.zeros(8)
    trace = np.zeros(8 * 8)
    rc = lib().orc_ieskf_update(omap.h, _p(body, C.c_float), len(body), C.byref(s), _p(Pc, C.c_double),
                                C.byref(mp), R, max_iter, limit, threads, _p(stats, C.c_double),
                                _p(trace, C.c_double), C.byref(sk))
    assert rc == 0
    out = (state_from_c(s), Pc, stats, trace.reshape(8, 8))
    return out + (state_from_c(sk),) if knn_state else out


def icp_align(src, dst, params=None, guess=None, threads=8, max_trace=64, want_aligned=False):
    params = params or default_icp_params()
    src = np.ascontiguousarray(src, dtype=np.float32)
    dst = np.ascontiguousarray(dst, dtype=np.float32)
    g = np.ascontiguousarray(np.eye(4, dtype=np.float32) if guess is None else guess, dtype=np.float32)
    T = np.zeros(16, np.float32)
    out = np.zeros(8)
    trace = np.zeros(20 * max_trace)
    aligned = np.empty_like(src) if want_aligned else None
    rc = lib().orc_icp_align(_p(src, C.c_float), len(src), _p(dst, C.c_float), len(dst), C.byref(params),
                             _p(g, C.c_float), _p(T, C.c_float), _p(out, C.c_double),
                             _p(aligned, C.c_float) if want_aligned else None, _p(trace, C.c_double),
                             max_trace, threads)
    assert rc == 0
    it = int(out[2])
    return dict(T=T.reshape(4, 4), fitness=out[0], converged=bool(out[1]), iterations=it, state=int(out[3]),
                is_valid=bool(out[4]), trace=trace.reshape(max_trace, 20)[:it], aligned=aligned)


class _TreeView:
    """Borrowed kd-tree handle (owned by an OracleDynMap)."""

    def __init__(self, h, owner):
        self.h, self._owner = h, owner


class OracleDynMap:
    """Incremental map restatement: ikd-Tree Add_Points / Delete_Point_Boxes and
    FAST-LIO map_incremental() semantics (oracle/lio_oracle.cpp DynMap)."""

    def __init__(self, xyz: np.ndarray):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        self.h = lib().orc_dmap_create(_p(xyz, C.c_float), len(xyz))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_dmap_free(self.h)
            self.h = None

    def num_ids(self):
        return int(lib().orc_dmap_num_ids(self.h))

    def size(self):
        return int(lib().orc_dmap_alive_count(self.h))

    def by_id(self):
        n = self.num_ids()
        xyz = np.empty((n, 3), np.float32)
        alive = np.empty(n, np.uint8)
        lib().orc_dmap_get(self.h, _p(xyz, C.c_float), _p(alive, C.c_uint8))
        return xyz, alive.astype(bool)

    def add(self, xyz, downsample, ds=0.5):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        return int(lib().orc_dmap_add(self.h, _p(xyz, C.c_float), len(xyz), int(downsample), C.c_float(ds)))

    def delete_boxes(self, boxes):
        b = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 6)
        return int(lib().orc_dmap_delete_boxes(self.h, _p(b, C.c_float), len(b)))

    def knn(self, q, k=5, range_sq=5.0):
        q = np.ascontiguousarray(q, dtype=np.float32).reshape(-1, 3)
        idx = np.empty((len(q), k), np.int32)
        d2 = np.empty((len(q), k), np.float32)
        assert lib().orc_dmap_knn(self.h, _p(q, C.c_float), len(q), k, C.c_float(range_sq), _p(idx, C.c_int32),
                                  _p(d2, C.c_float)) == 0
        return idx, d2

    def tree(self):
        """A map handle (the DynMap's kd-tree over its alive ids, same ids) for h_share_model /
        ieskf_update; valid until the DynMap changes."""
        return _TreeView(lib().orc_dmap_tree(self.h), self)

    def map_incremental(self, body, pose_knn24, pose24, fs=0.5, ds=0.5):
        body = np.ascontiguousarray(body, dtype=np.float32).reshape(-1, 3)
        pk = _pose32(pose_knn24)
        pf = _pose32(pose24)
        st = np.zeros(4, np.int64)
        lib().orc_map_incremental(self.h, _p(body, C.c_float), len(body), _p(pk, C.c_double), _p(pf, C.c_double),
                                  float(fs), C.c_float(ds), _p(st, C.c_int64))
        return dict(n_to_add=int(st[0]), n_no_downsample=int(st[1]), n_skipped=int(st[2]),
                    n_added_downsample=int(st[3]))


def voxel_grid(pts, leaf):
    """pcl::VoxelGrid (PCL 1.10) restatement; pts (n, stride) float32."""
    pts = np.ascontiguousarray(pts, dtype=np.float32)
    leaf3 = np.ascontiguousarray(np.broadcast_to(np.asarray(leaf, np.float32), 3))
    out = np.empty_like(pts)
    m = lib().orc_voxel_grid(_p(pts, C.c_float), len(pts), pts.shape[1], _p(leaf3, C.c_float), _p(out, C.c_float))
    assert m >= 0
    return out[:m].copy()


def submap_voxelize(clouds, poses, voxel_res):
    clouds = [np.ascontiguousarray(c, dtype=np.float32) for c in clouds]
    seg = np.zeros(len(clouds) + 1, np.int64)
    for k, c in enumerate(clouds):
        seg[k + 1] = seg[k] + len(c)
    pts = np.ascontiguousarray(np.concatenate(clouds))
    T = np.ascontiguousarray(np.stack([np.asarray(p, np.float64).reshape(4, 4) for p in poses]))
    out = np.empty_like(pts)
    m = lib().orc_submap_voxelize(_p(pts, C.c_float), _p(seg, C.c_int64), len(clouds), pts.shape[1],
                                  _p(T, C.c_double), C.c_float(voxel_res), _p(out, C.c_float))
    return out[:m].copy()


def preprocess(raw, imu_poses, end24, point_filter_num=4, blind=2.0, leaf=0.5, time_field=4):
    """Preprocess + UndistortPcl + downSizeFilterSurf restatement.  imu_poses: list of dicts."""
    raw = np.ascontiguousarray(raw, dtype=np.float32)
    P = np.zeros((max(len(imu_poses), 1), 22), np.float64)
    for k, p in enumerate(imu_poses):
        P[k] = np.concatenate([[p["offset_time"]], p["acc"], p["gyr"], p["vel"], p["pos"],
                               np.asarray(p["rot"], float).ravel()])
    e = _pose32(end24)
    out = np.empty_like(raw)
    m = lib().orc_preprocess(_p(raw, C.c_float), len(raw), raw.shape[1], point_filter_num, C.c_float(blind),
                             C.c_float(leaf), time_field, _p(P, C.c_double), len(imu_poses), _p(e, C.c_double),
                             _p(out, C.c_float))
    return out[:m].copy()
