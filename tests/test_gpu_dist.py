"""Multi-process sharded loop ICP with GPU-computed statistics.

tests/test_dist_gloo.py checks the exchange and the host combine with random
records on CPU; here every rank is a separate process that runs the HIP
correspondence + statistics kernels on its shard of the source (device 0 for
every rank: the one-GPU box) and all-gathers the real records through
lio_gpu.dist over torch.distributed (gloo: CPU tensors, so the ranks may share
the card).  Every rank must end with the transform, iteration count and score
of the single-process alignment, bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from lio_gpu import loop_closure as LC
from lio_gpu import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "fast-lio-sam_gps_amd")

RANK_CODE = r'''
import json, os, sys
sys.path.insert(0, r"%s")
import numpy as np
import torch.distributed as dist
from lio_gpu import dist as ld, loop_closure as LC, synth
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
src, dst, _ = synth.make_icp_pair(n_points=%d, seed=7, disp=(%f, %f))
lc = LC.LoopClosure(LC.LoopClosureConfig(), device=0)
if os.environ.get("LIO_TEST_EXCHANGE") == "shm":  # the C++ shared-memory exchange: no Python per pass
    lc.set_shard_shm(rank, world, "/lio_gpudist_%%s" %% os.environ["MASTER_PORT"], len(src))
else:
    cb = ld.make_allgather()
    lc.set_shard(rank, world, cb)
lc.setInputTarget(dst)
lc.setInputSource(src)
r = lc.align(keep_aligned=False)
dist.barrier()
print("RESULT " + json.dumps({"rank": rank, "T": np.asarray(r.T, np.float32).tobytes().hex(),
                              "iterations": int(r.iterations), "score": float(r.score).hex()}), flush=True)
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,disp,exchange", [(2, (0.3, 1.5), "gloo"), (3, (2.5, 4.0), "gloo"),
                                                  (2, (2.5, 4.0), "shm"), (3, (1.0, 3.0), "shm")])
def test_sharded_icp_multiprocess_gpu_records(world, disp, exchange):
    """exchange "gloo": the records through a ctypes callback into torch.distributed; "shm": the C++
    shared-memory exchange (lio_icp_set_shard_shm) — no Python call inside the alignment."""
    n = 60_000
    src, dst, _ = synth.make_icp_pair(n_points=n, seed=7, disp=disp)
    lc = LC.LoopClosure(LC.LoopClosureConfig(), device=0)
    lc.setInputTarget(dst)
    lc.setInputSource(src)
    ref = lc.align(keep_aligned=False)
    lc.close()
    code = RANK_CODE % (PKG, n, disp[0], disp[1])
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0", LIO_TEST_EXCHANGE=exchange)
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, o + e
            outs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = [json.loads(ln[7:]) for o in outs for ln in o.splitlines() if ln.startswith("RESULT ")]
    assert len(res) == world
    t_ref = np.asarray(ref.T, np.float32).tobytes().hex()
    for r in res:
        assert r["T"] == t_ref, f"rank {r['rank']}: transform differs from one process"
        assert r["iterations"] == ref.iterations
        assert r["score"] == float(ref.score).hex()
