"""Sharded loop ICP at C4 (500 k vs 500 k), the default PCL float order 2, `world` ranks emulated as threads on
one GPU with the device-side exchange (lio_icp_set_shard_device, the form RCCL uses; the all-gather emulated by
device copies on each rank's stream, as tests/test_gpu_icp.py::test_icp_device_exchange_emulated_ranks does).

    python scripts/icp_shard_profile.py WORLD [REPS] [DISP]

Prints ms per alignment for one rank alone and for the emulated ranks (which time-slice one card), checks every
rank's transform against the one-rank transform bit for bit.  Under `rocprofv3 --kernel-trace` the kernels of each
rank land on that rank's HIP stream: scripts/icp_shard_kernels.py splits the trace by stream and reports each
rank's per-pass kernel time (the figure the per-rank scaling model needs: the split work shrinks with WORLD, the
event walk and the exchanges do not)."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import torch  # noqa: E402

from lio_gpu import _capi, dist as ld  # noqa: E402
from lio_gpu import loop_closure as LC  # noqa: E402
from lio_gpu import synth  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
disp = (2.5, 4.0) if (len(sys.argv) <= 3 or sys.argv[3] == "B") else (0.3, 1.5)
src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321, disp=disp)

one = LC.LoopClosure(LC.LoopClosureConfig())
one.setInputSource(src)
one.setInputTarget(dst)
r1 = one.align(keep_aligned=False)
t0 = time.perf_counter()
for _ in range(reps):
    r1 = one.align(keep_aligned=False)
ms1 = (time.perf_counter() - t0) / reps * 1e3
T1 = np.array(list(r1.T), np.float32)
print(f"one rank: {ms1:.3f} ms per alignment, {r1.iterations} iterations, {one.fidelity_stats()}", flush=True)

n = ld.exchange_len(len(src), world)
dev = torch.device("cuda", 0)
sends = [torch.zeros(n, dtype=torch.float64, device=dev) for _ in range(world)]
recvs = [torch.zeros(n * world, dtype=torch.float64, device=dev) for _ in range(world)]
evs = [None] * world
bar = threading.Barrier(world)
calls = [0] * world


def make_cb(rank):
    def cb(send_p, nn, recv_p, stream, user):
        try:
            s = torch.cuda.ExternalStream(stream, device=dev)
            e = torch.cuda.Event()
            e.record(s)
            evs[rank] = e
            bar.wait()
            with torch.cuda.stream(s):
                for k in range(world):
                    s.wait_event(evs[k])
                    recvs[rank][k * nn:(k + 1) * nn].copy_(sends[k][:nn])
            s.synchronize()
            bar.wait()
            calls[rank] += 1
            return 0
        except Exception:
            import traceback

            traceback.print_exc()
            return -1

    return _capi.ALLGATHER_DEV_FN(cb)


cbs = [make_cb(r) for r in range(world)]
lcs = [LC.LoopClosure(LC.LoopClosureConfig()) for _ in range(world)]
res = [None] * world
times = [[] for _ in range(world)]


def run(rank):
    h = lcs[rank]._h
    _capi.check(_capi.lib().lio_icp_set_shard_device(h, rank, world, cbs[rank], None))
    lcs[rank].setInputSource(src)
    _capi.check(_capi.lib().lio_icp_set_exchange_buffers(h, sends[rank].data_ptr(), recvs[rank].data_ptr(), n))
    lcs[rank].setInputTarget(dst)
    for k in range(reps + 1):
        t = time.perf_counter()
        res[rank] = lcs[rank].align(keep_aligned=False)
        if k:
            times[rank].append((time.perf_counter() - t) * 1e3)


th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
[t.start() for t in th]
[t.join(timeout=600) for t in th]
for r in range(world):
    assert res[r] is not None, f"rank {r} did not finish"
    assert np.array_equal(np.array(list(res[r].T), np.float32), T1), f"rank {r}: transform differs from one rank"
    assert res[r].iterations == r1.iterations and res[r].score == r1.score
print(f"{world} emulated ranks (one GPU, time-sliced): {np.median([np.median(t) for t in times]):.3f} ms per alignment "
      f"(wall, all ranks sharing the card), exchanges per rank {calls[0] // (reps + 1)} per alignment, "
      f"fidelity {[lc.fidelity_stats() for lc in lcs][0]}; every rank bit-identical to one rank", flush=True)
