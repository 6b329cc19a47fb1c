"""Per-scan time decomposition of the IESKF update on the GPU box (diagnostics):
wall time per scan vs kernel time (HIP events) vs host solve time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene, m, scans = synth.make_config(cfg, n_scans=4)
dev = torch.device("cuda", 0)
d_scans = [torch.from_numpy(s.body).to(dev) for s in scans]
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build(m)
hm = F.HShareModelGPU(tree)
kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
P0 = synth.initial_cov()
states = [synth.initial_state(s.pos_init, s.rot_init) for s in scans]


def step(k):
    j = k % len(scans)
    hm.set_scan_device(d_scans[j].data_ptr(), len(scans[j].body))
    return kf.update_iterated_dyn_share_modified(states[j], P0)


for k in range(20):
    step(k)
torch.cuda.synchronize()
for rep in range(3):
    hm.reset_timing()
    hm.set_timing(True)
    N = 200
    solve = evals = knn = 0.0
    t0 = time.perf_counter()
    for k in range(N):
        x, P, st = step(k)
        solve += st["solve_ms"]
        evals += st["h_evals"]
        knn += st["knn_calls"]
    wall = (time.perf_counter() - t0) / N * 1e3
    hm.set_timing(False)
    t = hm.timing()
    kern = (t["knn_ms"] + t["reuse_ms"]) / N  # the sums are published by the last block (no finalize launch)
    print(f"rep{rep} wall_ms/scan={wall:.4f} kernels_ms/scan={kern:.4f} solve_ms/scan={solve / N:.4f} "
          f"other_ms/scan={wall - kern - solve / N:.4f} h_evals/scan={evals / N:.2f} knn/scan={knn / N:.2f}", flush=True)
# without timing events
t0 = time.perf_counter()
for k in range(200):
    step(k)
print(f"no-events wall_ms/scan={(time.perf_counter() - t0) / 200 * 1e3:.4f}")
# python/ctypes overhead floor: state conversion only
t0 = time.perf_counter()
for k in range(2000):
    s = F.state_to_c(states[0])
    F.state_from_c(s)
print(f"python state conversion us={(time.perf_counter() - t0) / 2000 * 1e6:.1f}")
