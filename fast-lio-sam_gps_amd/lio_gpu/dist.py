"""Multi-GPU plumbing for the sharded loop ICP (one process per GPU).

The ICP correspondence search shards the SOURCE cloud over ranks in whole
4096-point records (``lio_icp_shard_range``); per iteration every rank
all-gathers the per-record Umeyama statistics (20 doubles/record) and sums
them in record order (``lio_icp_combine``), so every rank — and every world
size — computes the bit-identical transform.  The exchange goes through
``torch.distributed`` (backend "nccl" = RCCL over xGMI on the GPU box, "gloo"
in the CPU tests): torch is plumbing here, the statistics are produced by the
HIP kernels behind the C-ABI.  SURVEY.md §8e.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import check, lib


def shard_range(n_source: int, rank: int, world: int):
    b, n = C.c_int64(), C.c_int64()
    check(lib().lio_icp_shard_range(n_source, rank, world, C.byref(b), C.byref(n)))
    return b.value, n.value


def combine(recv: np.ndarray, n_source: int, world: int) -> np.ndarray:
    recv = np.ascontiguousarray(recv, dtype=np.float64)
    out = np.zeros(17)
    check(lib().lio_icp_combine(recv.ctypes.data_as(C.POINTER(C.c_double)), n_source, world,
                                out.ctypes.data_as(C.POINTER(C.c_double))))
    return out


def allgather_numpy(send: np.ndarray, group=None, device=None) -> np.ndarray:
    """All-gather one float64 vector per rank (rank order) through torch.distributed."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = torch.from_numpy(np.ascontiguousarray(send, dtype=np.float64))
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy()


def make_allgather(group=None, device=None):
    """ctypes ``lio_allgather_fn`` doing the exchange with torch.distributed.

    ``device``: where the exchanged tensor lives.  RCCL ("nccl") only moves device tensors, so with
    that backend it defaults to the current CUDA device; gloo works on CPU tensors (None).
    A failing callback makes ``lio_icp_align`` return LIO_ERR_STATE on that rank while the other
    ranks wait inside the collective: the caller must then abort every rank (e.g. by raising,
    which ends the torchrun job), never retry the alignment alone.
    Keep the returned object alive while the ICP handle uses it.
    """
    import torch.distributed as dist

    if device is None and dist.get_backend(group) == "nccl":
        import torch

        device = torch.device("cuda", torch.cuda.current_device())

    def _cb(send_p, n, recv_p, user):
        try:
            send = np.ctypeslib.as_array(send_p, shape=(n,)).copy()
            res = allgather_numpy(send, group=group, device=device)
            recv = np.ctypeslib.as_array(recv_p, shape=(res.size,))
            recv[:] = res
            return 0
        except Exception:  # the C side turns a non-zero status into LIO_ERR_STATE
            import traceback

            traceback.print_exc()
            return -1

    return _capi.ALLGATHER_FN(_cb)


# the sharded float chains' messages (lio_seqsum.hpp): block sums ([0] the window's count; per chain at
# SEQ_TOT_HDR + 2 c nb_slot its 1024-element blocks' (double sum, sum |x|)) and event lists (header: n, overflow bits,
# increment totals, event counts, first elements; then per chain `slot` events of (increment prefix bits,
# position | value bits << 32))
SEQ_MAX_CHAINS, SEQ_TOT_HDR, SEQ_HDR_WORDS, SEQ_BLOCK = 9, 8, 32, 1024


def seq_shard_offsets(recv: np.ndarray, stride: int, nb_slot: int, rank: int, world: int, nch: int):
    """rank `rank`'s window of chains 0..nch-1 from every rank's block sums (lio_seq_shard_offsets, the device's
    seq_shard_offsets): (starting prefixes, drift variances, common floors, first global index, total)"""
    recv = np.ascontiguousarray(recv, dtype=np.float64)
    off0, var0 = np.zeros(nch), np.zeros(nch)
    fl = np.zeros(nch, np.int32)
    gn = np.zeros(2, np.int64)
    check(lib().lio_seq_shard_offsets(recv.ctypes.data_as(C.POINTER(C.c_double)), stride, nb_slot, rank, world, nch,
                                      off0.ctypes.data_as(C.POINTER(C.c_double)), var0.ctypes.data_as(C.POINTER(C.c_double)),
                                      fl.ctypes.data_as(C.POINTER(C.c_int32)), gn.ctypes.data_as(C.POINTER(C.c_int64))))
    return off0, var0, fl, int(gn[0]), int(gn[1])


def seq_shard_merge(recv: np.ndarray, stride: int, world: int, slot: int, chain: int, evs: int) -> dict:
    """chain `chain`'s global event lists from every rank's event message (lio_seq_shard_merge, the device's
    seq_shard_merge)"""
    recv = np.ascontiguousarray(recv, dtype=np.float64)
    pos, P, x = np.zeros(evs, np.int32), np.zeros(evs, np.uint64), np.zeros(evs, np.float32)
    info, ptot, x0 = np.zeros(3, np.int32), np.zeros(1, np.uint64), np.zeros(1, np.float32)
    check(lib().lio_seq_shard_merge(recv.ctypes.data_as(C.POINTER(C.c_double)), stride, world, slot, chain, evs,
                                    pos.ctypes.data_as(C.POINTER(C.c_int32)), P.ctypes.data_as(C.POINTER(C.c_uint64)),
                                    x.ctypes.data_as(C.POINTER(C.c_float)), info.ctypes.data_as(C.POINTER(C.c_int32)),
                                    ptot.ctypes.data_as(C.POINTER(C.c_uint64)), x0.ctypes.data_as(C.POINTER(C.c_float))))
    ne = int(info[0]) if info[2] == 0 else 0
    return dict(pos=pos[:ne], P=P[:ne], x=x[:ne], nev=int(info[0]), longest=int(info[1]), bad=int(info[2]),
                ptot=int(ptot[0]), x0=float(x0[0]))


def exchange_len(n_source: int, world: int) -> int:
    """doubles per rank of the device-side exchange (lio_icp_exchange_len)"""
    n = C.c_int64()
    check(lib().lio_icp_exchange_len(n_source, world, C.byref(n)))
    return n.value


class DeviceExchange:
    """Device-side record exchange for one rank (``lio_icp_set_shard_device``) over torch.distributed
    with the NCCL (= RCCL) backend: the send / recv buffers are torch tensors on this rank's GPU,
    handed to the ICP handle, and the callback runs ``all_gather_into_tensor`` on the handle's own
    HIP stream (``torch.cuda.ExternalStream``) — the records never leave the device and the handle
    waits once per pass for 17 sums.  Keep the object alive while the handle uses it."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.send = self.recv = None
        self.n = 0

        def _cb(send_p, n, recv_p, stream, user):
            try:
                assert send_p == self.send.data_ptr() and recv_p == self.recv.data_ptr() and n <= self.n
                with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device)):
                    dist.all_gather_into_tensor(self.recv[: n * self.world], self.send[:n], group=self.group)
                return 0
            except Exception:  # the C side turns a non-zero status into LIO_ERR_STATE
                import traceback

                traceback.print_exc()
                return -1

        self.fn = _capi.ALLGATHER_DEV_FN(_cb)

    def attach(self, handle, n_source: int):
        """(Re)size the buffers for a source of n_source points and hand them to the ICP handle."""
        import torch

        n = exchange_len(n_source, self.world)
        if n > self.n:
            self.send = torch.zeros(n, dtype=torch.float64, device=self.device)
            self.recv = torch.zeros(n * self.world, dtype=torch.float64, device=self.device)
            self.n = n
        check(lib().lio_icp_set_exchange_buffers(handle, self.send.data_ptr(), self.recv.data_ptr(), self.n))


# ---------------------------------------------------------------- C++ exchanges (no Python per pass)
def rccl_unique_id() -> bytes:
    """ncclGetUniqueId through the library's run-time-loaded librccl (rank 0 only)."""
    buf = (C.c_uint8 * 128)()
    check(lib().lio_rccl_unique_id(buf))
    return bytes(buf)


def broadcast_bytes(data: bytes | None, n: int, group=None) -> bytes:
    """rank 0's n bytes to every rank, once, through torch.distributed (set-up only, never per pass)."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.zeros(n, dtype=torch.uint8, device=dev)
    if dist.get_rank(group) == 0:
        t.copy_(torch.tensor(list(data), dtype=torch.uint8))
    dist.broadcast(t, src=0, group=group)
    return bytes(t.cpu().tolist())


def attach_rccl(handle, rank: int, world: int, group=None) -> None:
    """One RCCL communicator per rank created in C++ (lio_icp_set_shard_rccl): the unique id crosses
    torch.distributed once; every pass's all-gather is then enqueued by the library on the handle's stream."""
    uid = broadcast_bytes(rccl_unique_id() if rank == 0 else None, 128, group)
    buf = (C.c_uint8 * 128).from_buffer_copy(uid)
    check(lib().lio_icp_set_shard_rccl(handle, rank, world, buf))


def attach_shm(handle, rank: int, world: int, name: str, max_source_points: int, group=None) -> None:
    """The shared-memory exchange (lio_icp_set_shard_shm): rank 0 creates the segment, a barrier, the other
    ranks open it; every pass then exchanges in C++."""
    import torch.distributed as dist

    if rank == 0:
        check(lib().lio_icp_set_shard_shm(handle, rank, world, name.encode(), int(max_source_points)))
    dist.barrier(group)
    if rank != 0:
        check(lib().lio_icp_set_shard_shm(handle, rank, world, name.encode(), int(max_source_points)))
    dist.barrier(group)


class ShmExchange:
    """The bare shared-memory all-gather (lio_shm_exchange_*; host only): n doubles from every rank."""

    def __init__(self, name: str, rank: int, world: int, n: int, timeout_s: float | None = None):
        self._h = C.c_void_p()
        check(lib().lio_shm_exchange_open(name.encode(), rank, world, n, C.byref(self._h)))
        self.world = world
        if timeout_s is not None:
            check(lib().lio_shm_exchange_set_timeout(self._h, float(timeout_s)))

    def allgather(self, send: np.ndarray) -> np.ndarray:
        send = np.ascontiguousarray(send, dtype=np.float64)
        recv = np.empty(self.world * send.size)
        check(lib().lio_shm_exchange_allgather(self._h, send.ctypes.data_as(C.POINTER(C.c_double)), send.size,
                                               recv.ctypes.data_as(C.POINTER(C.c_double))))
        return recv

    def close(self):
        if self._h:
            lib().lio_shm_exchange_close(self._h)
            self._h = C.c_void_p()
