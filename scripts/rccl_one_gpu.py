"""Two ranks on ONE GPU over torch.distributed's NCCL backend (= RCCL): a plain all_gather_into_tensor,
then the sharded loop ICP with the device-side record exchange (lio_icp_set_shard_device +
lio_gpu.dist.DeviceExchange: the records all-gathered by RCCL on the ICP handle's stream), compared with
a single-rank alignment of the same pair.  Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29531 scripts/rccl_one_gpu.py
(RCCL may refuse two ranks on one device; the script then reports that and exits non-zero.)"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import dist as ldist  # noqa: E402
from lio_gpu import loop_closure as LC  # noqa: E402
from lio_gpu import synth  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), dtype=torch.float64, device="cuda")
    out = torch.empty(4 * world, dtype=torch.float64, device="cuda")
    dist.all_gather_into_tensor(out, t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_gather_into_tensor -> {out.tolist()}", flush=True)
    ok = True
    for disp in ((0.3, 1.5), (2.5, 4.0)):
        src, dst, _ = synth.make_icp_pair(n_points=200_000, seed=4321, disp=disp)
        ref = LC.LoopClosure(LC.LoopClosureConfig(), device=0)
        ref.setInputSource(src)
        ref.setInputTarget(dst)
        r1 = ref.align(keep_aligned=False)
        lc = LC.LoopClosure(LC.LoopClosureConfig(), device=0)
        ex = ldist.DeviceExchange()
        lc.set_shard_device(rank, world, ex)
        lc.setInputSource(src)
        lc.setInputTarget(dst)
        rn = lc.align(keep_aligned=False)
        same = (np.array_equal(np.asarray(r1.T), np.asarray(rn.T)) and r1.iterations == rn.iterations
                and r1.score == rn.score and r1.is_converged == rn.is_converged)
        ok &= same
        print(f"rank {rank} disp={disp}: 1 rank iters={r1.iterations} score={r1.score:.9f} | {world} ranks (RCCL device "
              f"exchange) iters={rn.iterations} score={rn.score:.9f} bit-identical={same}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
