#!/usr/bin/env python3
"""C3 map growth (bench.py's setup): per map_incremental call, the host wall time, the offered / added
counts and the grid geometry (a change means the call rebuilt the grid).  Diagnostics only."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import frontend as F, synth  # noqa: E402

n_grow = int(sys.argv[1]) if len(sys.argv) > 1 else 20
mp, L, sp, kind = synth.CONFIGS["C3"]
scene = synth.make_scene(L, 1234)
mappts = synth.sample_surface(scene, mp, 1234)
dev = torch.device("cuda", 0)
d_map = torch.from_numpy(mappts).to(dev)
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build_device(d_map.data_ptr(), len(mappts))
hm = F.HShareModelGPU(tree)
kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
P0 = synth.initial_cov()
grow = []
for k in range(n_grow):
    x = -0.15 * L + 1.85 + k * 3.7
    grow.append(synth.make_scan(scene, sp, kind, pos_gt=[x, 0.6 * np.sin(0.7 * k + 0.3), 0.0],
                                yaw_gt=0.05 * np.sin(0.3 * k + 0.2), seed=5099 + k))
d_grow = [torch.from_numpy(s.body).to(dev) for s in grow]
torch.cuda.synchronize()
print("grid0", tree.grid(), tree.stats(), flush=True)
for k, s in enumerate(grow):
    hm.set_scan_device(d_grow[k].data_ptr(), len(s.body))
    xg, _, _ = kf.update_iterated_dyn_share_modified(synth.initial_state(s.pos_init, s.rot_init), P0)
    g0 = str(tree.grid())
    ti = time.perf_counter()
    st = hm.map_incremental(synth.pose24(xg), 0.5)
    ms = (time.perf_counter() - ti) * 1e3
    g1 = str(tree.grid())
    print(f"call {k:2d} {ms:8.3f} ms  to_add {st['n_to_add']:6d} no_need {st['n_no_downsample']:6d} "
          f"size {tree.size()} geometry changed {g0 != g1} {tree.stats()}", flush=True)
