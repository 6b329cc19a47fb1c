"""ctypes declarations of include/lio_gpu.h and the loader for liblio_gpu.so.

The shared library is built in-tree (``make -C fast-lio-sam_gps_amd``) into
``lio_gpu/_lib/liblio_gpu.so``.  There is no fallback: if the library is
missing, :func:`lib` raises, and every compute entry point of the library
itself fails with ``LIO_ERR_NODEV`` when no gfx950 device is visible.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# LIO_GPU_LIB: load another build of the library (A/B diagnostics between builds)
LIB_PATH = os.environ.get("LIO_GPU_LIB") or os.path.join(HERE, "_lib", "liblio_gpu.so")

LIO_OK = 0
LIO_ERR_ARG = -1
LIO_ERR_HIP = -2
LIO_ERR_NODEV = -3
LIO_ERR_STATE = -4
LIO_ERR_NOMEM = -5
LIO_SUMS_LEN = 32
SUMS_HTH, SUMS_HTh, SUMS_NEFF, SUMS_RES, SUMS_HH = 0, 21, 27, 28, 29

# Every symbol include/lio_gpu.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = [
    "lio_device_count", "lio_last_error", "lio_build_info", "lio_abi_struct_sizes", "lio_alloc_count",
    "lio_map_create", "lio_map_destroy", "lio_map_set_params", "lio_map_build", "lio_map_build_device", "lio_map_size",
    "lio_map_get_points", "lio_map_get_grid", "lio_map_get_stats", "lio_map_num_ids", "lio_map_get_by_id", "lio_map_nearest_search", "lio_map_gather", "lio_map_add",
    "lio_map_add_device", "lio_map_delete_boxes", "lio_localmap_update", "lio_map_incremental",
    "lio_ctx_get_knn_pose", "lio_filter_create", "lio_filter_destroy", "lio_voxel_grid", "lio_submap_voxelize",
    "lio_preprocess", "lio_scan_preprocess", "lio_cloud2_decode", "lio_cloud2_encode", "lio_scan_preprocess_cloud2",
    "lio_pcd_write_binary", "lio_pcd_read", "lio_map_build_pcd",
    "lio_ctx_create", "lio_ctx_destroy", "lio_scan_set", "lio_scan_set_device", "lio_scan_bind_device", "lio_match",
    "lio_get_knn", "lio_get_planes", "lio_get_world", "lio_get_h_rows", "lio_ctx_knn_stats",
    "lio_ieskf_update", "lio_ctx_set_seed_scale", "lio_scan_get_undistorted", "lio_scan_keyframe_cloud",
    "lio_icp_create", "lio_icp_destroy", "lio_icp_set_target", "lio_icp_set_source", "lio_icp_set_shard",
    "lio_icp_set_shard_device", "lio_icp_exchange_len", "lio_icp_set_exchange_buffers",
    "lio_icp_align", "icp_align", "lio_icp_group_create", "lio_icp_group_destroy", "lio_icp_group_size",
    "lio_icp_group_uses_rccl", "lio_icp_group_set_target", "lio_icp_group_set_source", "lio_icp_group_align",
    "lio_icp_shard_range", "lio_icp_combine", "lio_icp_umeyama_pcl_float", "lio_icp_get_correspondences",
    "lio_ctx_set_timing", "lio_ctx_get_timing", "lio_ctx_reset_timing", "lio_icp_set_timing", "lio_icp_get_timing",
    "lio_icp_umeyama_pcl_float_order", "lio_icp_get_fidelity_stats", "lio_icp_set_fidelity_debug", "lio_seqsum6",
    "lio_map_set_test_limits", "lio_rccl_unique_id", "lio_icp_set_shard_rccl", "lio_icp_set_shard_shm",
    "lio_shm_exchange_open", "lio_shm_exchange_allgather", "lio_shm_exchange_close", "lio_shm_exchange_set_timeout",
    "lio_seq_shard_offsets", "lio_seq_shard_merge",
]


class LioError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lio_gpu error {code}: {msg}")
        self.code = code


class MapParams(C.Structure):
    _fields_ = [("cell_size", C.c_float), ("downsample_size", C.c_float), ("device", C.c_int),
                ("reserved", C.c_int)]


class MatchParams(C.Structure):
    _fields_ = [("knn_range_sq", C.c_float), ("plane_thr", C.c_float), ("s_coef", C.c_double),
                ("s_gate", C.c_double)]


class Pose(C.Structure):
    _fields_ = [("R", C.c_double * 9), ("t", C.c_double * 3), ("R_LI", C.c_double * 9), ("t_LI", C.c_double * 3),
                ("q", C.c_double * 4), ("q_LI", C.c_double * 4)]


class State(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("rot", C.c_double * 4), ("offset_R_L_I", C.c_double * 4),
                ("offset_T_L_I", C.c_double * 3), ("vel", C.c_double * 3), ("bg", C.c_double * 3),
                ("ba", C.c_double * 3), ("grav", C.c_double * 3)]


class IeskfParams(C.Structure):
    _fields_ = [("laser_point_cov", C.c_double), ("max_iteration", C.c_int), ("epsi", C.c_double)]


class IeskfStats(C.Structure):
    _fields_ = [("h_evals", C.c_int), ("knn_calls", C.c_int), ("converged", C.c_int), ("n_eff", C.c_int),
                ("res_mean", C.c_double), ("solve_ms", C.c_double), ("wall_ms", C.c_double),
                ("launch_ms", C.c_double), ("wait_ms", C.c_double)]


class IcpParams(C.Structure):
    _fields_ = [("max_corr_dist", C.c_double), ("trans_eps", C.c_double), ("fitness_eps", C.c_double),
                ("max_iter", C.c_int), ("rot_eps", C.c_double), ("score_threshold", C.c_double),
                ("cell_size", C.c_float), ("device", C.c_int), ("umeyama_float", C.c_int)]


class IcpResult(C.Structure):
    _fields_ = [("is_valid", C.c_int), ("is_converged", C.c_int), ("score", C.c_double), ("T", C.c_float * 16),
                ("iterations", C.c_int), ("state", C.c_int), ("last_mse", C.c_double), ("last_corr", C.c_int64)]


class LocalMap(C.Structure):
    _fields_ = [("vertex_min", C.c_float * 3), ("vertex_max", C.c_float * 3), ("initialized", C.c_int)]


class IncrementalStats(C.Structure):
    _fields_ = [("n_to_add", C.c_int64), ("n_no_downsample", C.c_int64), ("n_skipped", C.c_int64),
                ("n_added_downsample", C.c_int64)]


class ImuPose(C.Structure):
    _fields_ = [("offset_time", C.c_double), ("acc", C.c_double * 3), ("gyr", C.c_double * 3), ("vel", C.c_double * 3),
                ("pos", C.c_double * 3), ("rot", C.c_double * 9)]


class ScanPrepParams(C.Structure):
    _fields_ = [("point_filter_num", C.c_int), ("blind", C.c_float), ("filter_size_surf", C.c_float),
                ("time_field", C.c_int)]


class CloudField(C.Structure):
    _fields_ = [("offset", C.c_int32), ("datatype", C.c_int32), ("scale", C.c_float)]


class KernelTiming(C.Structure):
    _fields_ = [("knn_launches", C.c_int64), ("knn_ms", C.c_double), ("reuse_launches", C.c_int64),
                ("reuse_ms", C.c_double),
                ("icp_launches", C.c_int64), ("icp_ms", C.c_double), ("near_launches", C.c_int64),
                ("near_ms", C.c_double), ("far_launches", C.c_int64), ("far_ms", C.c_double),
                ("plane_launches", C.c_int64), ("plane_ms", C.c_double),
                ("icp_nn_launches", C.c_int64), ("icp_nn_ms", C.c_double)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.c_void_p)
# lio_allgather_dev_fn(d_send, n, d_recv, stream, user): device pointers, enqueue on `stream`
ALLGATHER_DEV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p)

_lib = None

fp = C.POINTER(C.c_float)
dp = C.POINTER(C.c_double)
vp = C.c_void_p


def _declare(L):
    sig = {
        "lio_device_count": (C.c_int, []),
        "lio_alloc_count": (C.c_int64, []),
        "lio_last_error": (C.c_char_p, []),
        "lio_build_info": (C.c_char_p, []),
        "lio_abi_struct_sizes": (C.c_int, [C.POINTER(C.c_int64), C.c_int]),
        "lio_map_create": (C.c_int, [C.POINTER(MapParams), C.POINTER(vp)]),
        "lio_map_destroy": (C.c_int, [vp]),
        "lio_map_set_params": (C.c_int, [vp, C.POINTER(MapParams)]),
        "lio_map_build": (C.c_int, [vp, fp, C.c_int64]),
        "lio_map_build_device": (C.c_int, [vp, vp, C.c_int64]),
        "lio_map_size": (C.c_int64, [vp]),
        "lio_map_get_points": (C.c_int, [vp, fp]),
        "lio_map_get_grid": (C.c_int, [vp, dp]),
        "lio_map_get_stats": (C.c_int, [vp, C.POINTER(C.c_int64)]),
        "lio_map_set_test_limits": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "lio_rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "lio_icp_set_shard_rccl": (C.c_int, [vp, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
        "lio_icp_set_shard_shm": (C.c_int, [vp, C.c_int, C.c_int, C.c_char_p, C.c_int64]),
        "lio_shm_exchange_open": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int64, C.POINTER(vp)]),
        "lio_shm_exchange_allgather": (C.c_int, [vp, dp, C.c_int64, dp]),
        "lio_shm_exchange_close": (C.c_int, [vp]),
        "lio_shm_exchange_set_timeout": (C.c_int, [vp, C.c_double]),
        "lio_seq_shard_offsets": (C.c_int, [dp, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, dp, dp, C.POINTER(C.c_int32),
                                            C.POINTER(C.c_int64)]),
        "lio_seq_shard_merge": (C.c_int, [dp, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int64, C.POINTER(C.c_int32),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_float), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_float)]),
        "lio_map_num_ids": (C.c_int64, [vp]),
        "lio_map_get_by_id": (C.c_int, [vp, fp, C.POINTER(C.c_uint8)]),
        "lio_map_nearest_search": (C.c_int, [vp, fp, C.c_int64, C.c_int, C.c_float, C.POINTER(C.c_int32), fp]),
        "lio_map_gather": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int64, fp]),
        "lio_map_add": (C.c_int, [vp, fp, C.c_int64, C.c_int, C.POINTER(C.c_int64)]),
        "lio_map_add_device": (C.c_int, [vp, vp, C.c_int64, C.c_int, C.POINTER(C.c_int64)]),
        "lio_map_delete_boxes": (C.c_int, [vp, fp, C.c_int, C.POINTER(C.c_int64)]),
        "lio_localmap_update": (C.c_int, [C.POINTER(LocalMap), dp, C.c_double, C.c_float, C.c_float, fp,
                                          C.POINTER(C.c_int)]),
        "lio_map_incremental": (C.c_int, [vp, C.POINTER(Pose), C.c_double, C.POINTER(IncrementalStats)]),
        "lio_ctx_get_knn_pose": (C.c_int, [vp, C.POINTER(Pose)]),
        "lio_cloud2_decode": (C.c_int, [vp, vp, C.c_int64, C.c_int32, C.c_int, C.POINTER(CloudField), C.c_int, fp]),
        "lio_cloud2_encode": (C.c_int, [vp, fp, C.c_int64, C.c_int, C.POINTER(CloudField), C.c_int, C.c_int32, vp]),
        "lio_scan_preprocess_cloud2": (C.c_int, [vp, vp, C.c_int64, C.c_int32, C.c_int, C.POINTER(CloudField),
                                                 C.POINTER(ScanPrepParams), C.POINTER(ImuPose), C.c_int,
                                                 C.POINTER(Pose), C.POINTER(C.c_int64)]),
        "lio_pcd_write_binary": (C.c_int, [C.c_char_p, fp, C.c_int64, C.c_int, C.POINTER(C.c_char_p)]),
        "lio_pcd_read": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_char_p), C.c_int, fp, C.c_int64,
                                   C.POINTER(C.c_int64)]),
        "lio_map_build_pcd": (C.c_int, [vp, C.c_char_p]),
        "lio_filter_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "lio_filter_destroy": (C.c_int, [vp]),
        "lio_voxel_grid": (C.c_int, [vp, fp, C.c_int64, C.c_int, fp, fp, C.POINTER(C.c_int64)]),
        "lio_submap_voxelize": (C.c_int, [vp, fp, C.POINTER(C.c_int64), C.c_int, C.c_int, dp, C.c_float, fp,
                                          C.POINTER(C.c_int64)]),
        "lio_preprocess": (C.c_int, [vp, fp, C.c_int64, C.c_int, C.POINTER(ScanPrepParams), C.POINTER(ImuPose), C.c_int,
                                     C.POINTER(Pose), fp, C.POINTER(C.c_int64)]),
        "lio_scan_preprocess": (C.c_int, [vp, fp, C.c_int64, C.c_int, C.POINTER(ScanPrepParams), C.POINTER(ImuPose),
                                          C.c_int, C.POINTER(Pose), C.POINTER(C.c_int64)]),
        "lio_ctx_create": (C.c_int, [vp, C.POINTER(MatchParams), C.POINTER(vp)]),
        "lio_ctx_destroy": (C.c_int, [vp]),
        "lio_scan_set": (C.c_int, [vp, fp, C.c_int64]),
        "lio_scan_set_device": (C.c_int, [vp, vp, C.c_int64]),
        "lio_scan_bind_device": (C.c_int, [vp, vp, C.c_int64]),
        "lio_match": (C.c_int, [vp, C.POINTER(Pose), C.c_int, dp]),
        "lio_get_knn": (C.c_int, [vp, C.POINTER(C.c_int32), fp]),
        "lio_get_planes": (C.c_int, [vp, fp, C.POINTER(C.c_uint8)]),
        "lio_get_world": (C.c_int, [vp, fp]),
        "lio_get_h_rows": (C.c_int, [vp, dp, C.c_int64, C.POINTER(C.c_int64)]),
        "lio_ctx_knn_stats": (C.c_int, [vp, C.POINTER(Pose), dp, C.POINTER(C.c_int32)]),
        "lio_ieskf_update": (C.c_int, [vp, C.POINTER(State), dp, C.POINTER(IeskfParams), C.POINTER(IeskfStats)]),
        "lio_ctx_set_seed_scale": (C.c_int, [vp, C.c_float]),
        "lio_scan_get_undistorted": (C.c_int, [vp, fp, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
        "lio_scan_keyframe_cloud": (C.c_int, [vp, C.POINTER(Pose), dp, fp, C.c_int64, C.POINTER(C.c_int64)]),
        "lio_icp_create": (C.c_int, [C.POINTER(IcpParams), C.POINTER(vp)]),
        "lio_icp_destroy": (C.c_int, [vp]),
        "lio_icp_set_target": (C.c_int, [vp, fp, C.c_int64]),
        "lio_icp_set_source": (C.c_int, [vp, fp, C.c_int64]),
        "lio_icp_set_shard": (C.c_int, [vp, C.c_int, C.c_int, ALLGATHER_FN, vp]),
        "lio_icp_set_shard_device": (C.c_int, [vp, C.c_int, C.c_int, ALLGATHER_DEV_FN, vp]),
        "lio_icp_exchange_len": (C.c_int, [C.c_int64, C.c_int, C.POINTER(C.c_int64)]),
        "lio_icp_set_exchange_buffers": (C.c_int, [vp, vp, vp, C.c_int64]),
        "lio_icp_align": (C.c_int, [vp, fp, C.POINTER(IcpResult), fp]),
        "lio_icp_get_correspondences": (C.c_int, [vp, C.POINTER(C.c_int32), fp]),
        "icp_align": (C.c_int, [fp, C.c_int64, fp, C.c_int64, C.POINTER(IcpParams), C.c_int, fp, dp,
                                C.POINTER(C.c_int), C.POINTER(C.c_int), fp]),
        "lio_icp_group_create": (C.c_int, [C.POINTER(IcpParams), C.c_int, C.POINTER(C.c_int), C.POINTER(vp)]),
        "lio_icp_group_destroy": (C.c_int, [vp]),
        "lio_icp_group_size": (C.c_int, [vp]),
        "lio_icp_group_uses_rccl": (C.c_int, [vp]),
        "lio_icp_group_set_target": (C.c_int, [vp, fp, C.c_int64]),
        "lio_icp_group_set_source": (C.c_int, [vp, fp, C.c_int64]),
        "lio_icp_group_align": (C.c_int, [vp, fp, C.POINTER(IcpResult), fp]),
        "lio_icp_shard_range": (C.c_int, [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "lio_icp_combine": (C.c_int, [dp, C.c_int64, C.c_int, dp]),
        "lio_icp_umeyama_pcl_float": (C.c_int, [fp, fp]),
        "lio_icp_umeyama_pcl_float_order": (C.c_int, [fp, C.c_int, fp]),
        "lio_icp_get_fidelity_stats": (C.c_int, [vp, C.POINTER(C.c_int64)]),
        "lio_icp_set_fidelity_debug": (C.c_int, [vp, C.c_int, C.c_int64]),
        "lio_seqsum6": (C.c_int, [C.c_int, fp, C.c_int64, C.c_int, fp, C.POINTER(C.c_int)]),
        "lio_ctx_set_timing": (C.c_int, [vp, C.c_int]),
        "lio_ctx_get_timing": (C.c_int, [vp, C.POINTER(KernelTiming)]),
        "lio_ctx_reset_timing": (C.c_int, [vp]),
        "lio_icp_set_timing": (C.c_int, [vp, C.c_int]),
        "lio_icp_get_timing": (C.c_int, [vp, C.POINTER(KernelTiming)]),
    }
    ab = bool(os.environ.get("LIO_GPU_LIB"))  # an older build for A/B timing may lack newer entry points
    for name, (res, args) in sig.items():
        if ab and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def _share_torch_hip_runtime():
    """One HIP runtime per process.

    PyTorch-ROCm bundles its own libamdhip64.so.7 (+ HSA runtime) under
    torch/lib; ours links /opt/rocm's under the same soname, so whichever loads
    first serves both, and torch cannot see the GPU through the other one
    ("No HIP GPUs are available").  When torch is installed, load its runtime
    first (without importing torch) so that device pointers from torch tensors
    (lio_scan_bind_device) and our kernels share one runtime.  A process
    without torch (the C++ host) uses /opt/rocm's.
    """
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        hip = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(hip):
            C.CDLL(hip, mode=C.RTLD_GLOBAL)
            return


def lib():
    """Load liblio_gpu.so (raises if it was not built — there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C fast-lio-sam_gps_amd` "
                              "(or __graft_entry__.build()); lio_gpu has no CPU path")
        _share_torch_hip_runtime()
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _check_abi(L)
        _lib = L
    return _lib


# the ctypes mirrors of lio_abi_struct_sizes' structs, in its order
_ABI_STRUCTS = ("MapParams", "MatchParams", "Pose", "State", "IeskfParams", "IeskfStats", "IcpParams", "IcpResult",
                "LocalMap", "IncrementalStats", "ImuPose", "ScanPrepParams", "CloudField", "KernelTiming")


def _check_abi(L):
    """Refuse a library whose public structs differ from these mirrors: an output struct of another size
    overruns the caller's buffer (how round 4's LIO_GPU_LIB A/B against a round-2 build corrupted the heap:
    its lio_kernel_timing carried an extra finalize pair, 128 bytes written into a 112-byte ctypes struct)."""
    n = int(L.lio_abi_struct_sizes(None, 0))
    sizes = (C.c_int64 * n)()
    L.lio_abi_struct_sizes(sizes, n)
    mine = [C.sizeof(globals()[k]) for k in _ABI_STRUCTS]
    if n != len(mine) or list(sizes) != mine:
        raise ImportError(f"{LIB_PATH}: ABI mismatch with lio_gpu/_capi.py — library struct sizes {list(sizes)}, "
                          f"binding {mine} ({', '.join(_ABI_STRUCTS)})")


def check(rc):
    if rc != LIO_OK:
        msg = lib().lio_last_error()
        raise LioError(rc, msg.decode() if msg else "")
    return rc
