"""Host mirror of ``LoopClosure`` (/root/reference/fast_lio_sam/include/loop_closure.h:21-72).

Only the ★ hot-path member ``icpAlignment`` (loop_closure.cpp:69-92) is backed
by the GPU; it keeps the class surface: configuration as in the constructor
(loop_closure.cpp:3-14), ``RegistrationOutput`` as returned value, the aligned
cloud kept for ``getFinalAlignedCloud`` (loop_closure.cpp:73,81,139-142).
Sharding over ranks (one process per GPU) plugs in through
:func:`lio_gpu.dist.make_allgather` — see include/lio_gpu.h lio_icp_set_shard.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import _capi
from ._capi import check, lib


@dataclasses.dataclass
class LoopClosureConfig:  # loop_closure.h:21-29, values from fast_lio_sam.cpp:64-80 + config.yaml
    num_submap_keyframes_: int = 5
    voxel_res_: float = 0.3
    loop_detection_radius_: float = 35.0
    loop_detection_timediff_threshold_: float = 30.0
    icp_score_threshold_: float = 1.5
    icp_max_corr_dist_: float = 52.5  # 1.5 * loop_detection_radius_ (fast_lio_sam.cpp:73)


@dataclasses.dataclass
class PosePcd:  # pose_pcd.hpp:7-19 (the fields setSrcAndDstCloud reads)
    pcd_: np.ndarray  # PointXYZI rows (x, y, z, intensity), float32
    pose_corrected_eig_: np.ndarray = dataclasses.field(default_factory=lambda: np.eye(4))
    pose_eig_: np.ndarray = dataclasses.field(default_factory=lambda: np.eye(4))
    timestamp_: float = 0.0
    idx_: int = 0


@dataclasses.dataclass
class RegistrationOutput:  # loop_closure.h:31-37
    is_valid_: bool = False
    is_converged_: bool = False
    score_: float = float(np.finfo(np.float64).max)
    pose_between_eig_: np.ndarray = dataclasses.field(default_factory=lambda: np.eye(4))
    iterations: int = 0
    state: int = 0


def _xyz(cloud) -> np.ndarray:
    """xyz columns of a cloud given as (n, 3) or PointXYZI-like (n, >= 3) rows."""
    a = np.asarray(cloud, dtype=np.float32)
    return a.reshape(-1, 3) if a.ndim == 1 else a[:, :3]


# lio_icp_params.umeyama_float: PCL's float Umeyama (TransformationEstimationSVD<PointXYZI, PointXYZI,
# float>, loop_closure.h:42) in a summation order — 1 sequential-order restatement, 2 the Eigen 3.3 GEMM
# model (32 KiB L1; THE DEFAULT: the reference's arithmetic), 3 as 2 with 48 KiB — or DOUBLE_STATS, the
# opt-in double statistics (faster, 1.2-1.9e-4 from the float orders at C4: outside the 1e-5 bar)
FIDELITY_ORDER = 2
DOUBLE_STATS = -1


def icp_params(config: LoopClosureConfig, cell_size: float = 1.0, device: int = 0,
               umeyama_float: int = FIDELITY_ORDER) -> _capi.IcpParams:
    # setTransformationEpsilon(0.01), setEuclideanFitnessEpsilon(0.01), setMaximumIterations(50)
    return _capi.IcpParams(config.icp_max_corr_dist_, 0.01, 0.01, 50, 0.0, config.icp_score_threshold_,
                           cell_size, device, int(umeyama_float))


class LoopClosure:
    def __init__(self, config: LoopClosureConfig, cell_size: float = 1.0, device: int = 0,
                 umeyama_float: int = FIDELITY_ORDER):
        """umeyama_float: 1..3 a float order of pcl::umeyama (default 2, the reference's arithmetic; sharded
        ranks all-gather their correspondence ids and give the one-rank transform bit for bit);
        DOUBLE_STATS (-1) the opt-in double statistics."""
        self.config_ = config
        self._p = icp_params(config, cell_size, device, umeyama_float)
        self._h = C.c_void_p()
        check(lib().lio_icp_create(C.byref(self._p), C.byref(self._h)))
        self.aligned_ = np.zeros((0, 3), np.float32)
        self._shard = (0, 1)
        self._cb = None

    def set_shard(self, rank: int, world: int, allgather=None):
        """Shard the source over ``world`` ranks; ``allgather`` from lio_gpu.dist.make_allgather
        (host-side exchange: the records pass through host memory)."""
        self._cb = allgather
        self._dx = None
        fn = allgather if allgather is not None else _capi.ALLGATHER_FN()
        check(lib().lio_icp_set_shard(self._h, rank, world, fn, None))
        self._shard = (rank, world)

    def set_shard_device(self, rank: int, world: int, exchange):
        """Shard the source over ``world`` ranks with the device-side exchange (``exchange``: a
        lio_gpu.dist.DeviceExchange; torch.distributed NCCL = RCCL backend)."""
        self._cb = None
        self._dx = exchange
        check(lib().lio_icp_set_shard_device(self._h, rank, world, exchange.fn, None))
        self._shard = (rank, world)

    def set_shard_rccl(self, rank: int, world: int, group=None):
        """Shard the source over ``world`` ranks with a per-rank RCCL communicator created in C++
        (lio_icp_set_shard_rccl): the all-gather of every pass is enqueued by the library, no Python."""
        from . import dist as ld

        self._cb = None
        self._dx = None
        ld.attach_rccl(self._h, rank, world, group)
        self._shard = (rank, world)

    def set_shard_shm(self, rank: int, world: int, name: str, max_source_points: int, group=None):
        """Shard over ranks on ONE node through the C++ shared-memory exchange (lio_icp_set_shard_shm)."""
        from . import dist as ld

        self._cb = None
        self._dx = None
        ld.attach_shm(self._h, rank, world, name, max_source_points, group)
        self._shard = (rank, world)

    def set_timing(self, on: bool):
        check(lib().lio_icp_set_timing(self._h, 1 if on else 0))

    def fidelity_stats(self) -> dict:
        """float fidelity modes: seqsum verification re-passes, serial fallbacks, events of the last pass
        (max over chains), passes run — since the handle was created"""
        out = (C.c_int64 * 4)()
        check(lib().lio_icp_get_fidelity_stats(self._h, out))
        return dict(repasses=out[0], serial=out[1], events=out[2], passes=out[3])

    def set_fidelity_debug(self, flags: int = 0, evcap: int = 0):
        check(lib().lio_icp_set_fidelity_debug(self._h, int(flags), int(evcap)))

    def timing(self) -> dict:
        t = _capi.KernelTiming()
        check(lib().lio_icp_get_timing(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in _capi.KernelTiming._fields_}

    def setInputTarget(self, dst: np.ndarray):
        d = np.ascontiguousarray(_xyz(dst), dtype=np.float32)
        check(lib().lio_icp_set_target(self._h, d.ctypes.data_as(C.POINTER(C.c_float)), len(d)))

    def setInputSource(self, src: np.ndarray):
        s = np.ascontiguousarray(_xyz(src), dtype=np.float32)
        check(lib().lio_icp_set_source(self._h, s.ctypes.data_as(C.POINTER(C.c_float)), len(s)))
        self._ns = len(s)
        if getattr(self, "_dx", None) is not None:
            self._dx.attach(self._h, len(s))

    def align(self, guess: np.ndarray | None = None, keep_aligned: bool = True):
        res = _capi.IcpResult()
        g = None if guess is None else np.ascontiguousarray(guess, dtype=np.float32).reshape(16)
        out = None
        if keep_aligned:
            rank, world = self._shard
            nsup = (self._ns + 4095) // 4096
            b = min(nsup * rank // world * 4096, self._ns)
            e = min(nsup * (rank + 1) // world * 4096, self._ns)
            out = np.empty((max(e - b, 0), 3), np.float32)
        check(lib().lio_icp_align(self._h, None if g is None else g.ctypes.data_as(C.POINTER(C.c_float)),
                                  C.byref(res), None if out is None else out.ctypes.data_as(C.POINTER(C.c_float))))
        if out is not None:
            self.aligned_ = out
        return res

    def correspondences(self):
        """1-NN (target index, float d2) of every source point of this rank's shard in the
        last pass (after align(): the getFitnessScore pass over the aligned cloud)."""
        rank, world = self._shard
        nsup = (self._ns + 4095) // 4096
        b = min(nsup * rank // world * 4096, self._ns)
        e = min(nsup * (rank + 1) // world * 4096, self._ns)
        ids = np.empty(max(e - b, 0), np.int32)
        d2 = np.empty(max(e - b, 0), np.float32)
        check(lib().lio_icp_get_correspondences(self._h, ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                                d2.ctypes.data_as(C.POINTER(C.c_float))))
        return ids, d2

    def fetchClosestKeyframeIdx(self, front_keyframe: PosePcd, keyframes) -> int:
        """loop_closure.cpp:18-40: among keyframes[0 .. size-2], the closest (translation of
        pose_corrected_eig_) within loop_detection_radius_ whose timestamp is more than
        loop_detection_timediff_threshold_ older; -1 if none."""
        radi = self.config_.loop_detection_radius_
        shortest = radi * 3.0
        closest = -1
        p = np.asarray(front_keyframe.pose_corrected_eig_, np.float64)[:3, 3]
        for kf in keyframes[:len(keyframes) - 1]:
            d = float(np.linalg.norm(np.asarray(kf.pose_corrected_eig_, np.float64)[:3, 3] - p))
            if radi > d and self.config_.loop_detection_timediff_threshold_ < (front_keyframe.timestamp_ - kf.timestamp_):
                if d < shortest:
                    shortest = d
                    closest = kf.idx_
        return closest

    def performLoopClosure(self, query_keyframe: PosePcd, keyframes, closest_keyframe_idx: int | None = None,
                           submap_range: int | None = None) -> RegistrationOutput:
        """loop_closure.cpp:95-126: submaps around the query and the closest keyframe
        (num_submap_keyframes_, voxel_res_), then icpAlignment(src, dst)."""
        if closest_keyframe_idx is None:
            closest_keyframe_idx = self.fetchClosestKeyframeIdx(query_keyframe, keyframes)
        self.closest_keyframe_idx_ = closest_keyframe_idx
        if closest_keyframe_idx < 0:
            return RegistrationOutput()
        rng = self.config_.num_submap_keyframes_ if submap_range is None else submap_range
        self.src_cloud_, self.dst_cloud_ = self.setSrcAndDstCloud(keyframes, query_keyframe.idx_, closest_keyframe_idx,
                                                                  rng, self.config_.voxel_res_)
        return self.icpAlignment(self.src_cloud_, self.dst_cloud_)

    def setSrcAndDstCloud(self, keyframes, src_idx: int, dst_idx: int, submap_range: int, voxel_res: float):
        """loop_closure.cpp:42-67 on the GPU: per side, transformPcd of keyframes
        [idx - range, idx + range] (skipping i >= keyframes.size() - 1: the newest keyframe
        never enters a submap, :54/:62), concatenated, voxelizePcd(voxel_res)."""
        from .filters import VoxelGrid, voxelize_submap

        if getattr(self, "_vg", None) is None:
            self._vg = VoxelGrid(voxel_res, device=self._p.device)

        def side(center):
            clouds, poses = [], []
            for i in range(center - submap_range, center + submap_range + 1):
                if 0 <= i < len(keyframes) - 1:
                    clouds.append(np.asarray(keyframes[i].pcd_, np.float32).reshape(-1, 4))
                    poses.append(keyframes[i].pose_corrected_eig_)
            if not clouds:
                return np.zeros((0, 4), np.float32)
            return voxelize_submap(clouds, poses, voxel_res, self._vg)

        return side(src_idx), side(dst_idx)

    def icpAlignment(self, src: np.ndarray, dst: np.ndarray) -> RegistrationOutput:
        """loop_closure.cpp:69-92: align src to dst; valid iff converged and score < threshold."""
        out = RegistrationOutput()
        self.aligned_ = np.zeros((0, 3), np.float32)
        self.setInputSource(src)
        self.setInputTarget(dst)
        res = self.align()
        out.score_ = res.score
        out.iterations = res.iterations
        out.state = res.state
        if res.is_converged and res.score < self.config_.icp_score_threshold_:
            out.is_valid_ = True
            out.is_converged_ = True
            out.pose_between_eig_ = np.array(list(res.T), dtype=np.float32).reshape(4, 4).astype(np.float64)
        self.last_result = res
        return out

    def getFinalAlignedCloud(self) -> np.ndarray:
        return self.aligned_

    def close(self):
        if self._h:
            lib().lio_icp_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LoopClosureGroup:
    """Single-process multi-GPU loop ICP (``lio_icp_group``): one handle per device, the source
    sharded, the per-iteration messages (records; in the PCL float modes also the windows' chain block sums,
    event lists and depth blocks) all-gathered over RCCL (or through host memory with
    ``LIO_ICP_EXCHANGE=host`` / a device listed twice).  Same results as :class:`LoopClosure`, bit
    for bit."""

    def __init__(self, config: LoopClosureConfig, n_gpus: int, devices=None, cell_size: float = 1.0,
                 umeyama_float: int = FIDELITY_ORDER):
        self.config_ = config
        self._p = icp_params(config, cell_size, 0 if devices is None else int(devices[0]), umeyama_float)
        self._h = C.c_void_p()
        devs = None
        if devices is not None:
            devs = (C.c_int * n_gpus)(*[int(d) for d in devices])
        check(lib().lio_icp_group_create(C.byref(self._p), int(n_gpus), devs, C.byref(self._h)))
        self.n_gpus = int(n_gpus)
        self._ns = 0

    @property
    def uses_rccl(self) -> bool:
        return bool(lib().lio_icp_group_uses_rccl(self._h))

    def setInputTarget(self, dst: np.ndarray):
        d = np.ascontiguousarray(_xyz(dst))
        check(lib().lio_icp_group_set_target(self._h, d.ctypes.data_as(C.POINTER(C.c_float)), len(d)))

    def setInputSource(self, src: np.ndarray):
        s = np.ascontiguousarray(_xyz(src))
        self._ns = len(s)
        check(lib().lio_icp_group_set_source(self._h, s.ctypes.data_as(C.POINTER(C.c_float)), len(s)))

    def align(self, guess: np.ndarray | None = None, keep_aligned: bool = True):
        res = _capi.IcpResult()
        g = None if guess is None else np.ascontiguousarray(guess, dtype=np.float32).reshape(16)
        out = np.empty((self._ns, 3), np.float32) if keep_aligned else None
        check(lib().lio_icp_group_align(self._h, None if g is None else g.ctypes.data_as(C.POINTER(C.c_float)),
                                        C.byref(res), None if out is None else out.ctypes.data_as(C.POINTER(C.c_float))))
        if out is not None:
            self.aligned_ = out
        return res

    def close(self):
        if self._h:
            lib().lio_icp_group_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
