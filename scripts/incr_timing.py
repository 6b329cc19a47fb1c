"""map_incremental timing on a C3-size map (diagnostics; run under rocprofv3 for the kernel split)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
nscan = int(sys.argv[2]) if len(sys.argv) > 2 else 12
scene, m, scans = synth.make_config(cfg, n_scans=nscan)
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build(m)
hm = F.HShareModelGPU(tree)
kf = F.EsekfGPU(hm)
P0 = synth.initial_cov()
t_upd = t_inc = 0.0
for k, sc in enumerate(scans):
    hm.set_scan(sc.body)
    t0 = time.perf_counter()
    x, P, st = kf.update_iterated_dyn_share_modified(synth.initial_state(sc.pos_init, sc.rot_init), P0)
    t1 = time.perf_counter()
    s = hm.map_incremental(synth.pose24(x), 0.5)
    t2 = time.perf_counter()
    if k >= 2:
        t_upd += t1 - t0
        t_inc += t2 - t1
    print(k, s, tree.size(), tree.num_ids(), f"upd_ms={(t1 - t0) * 1e3:.3f} inc_ms={(t2 - t1) * 1e3:.3f}", flush=True)
n = max(nscan - 2, 1)
print(f"mean upd_ms={t_upd / n * 1e3:.3f} inc_ms={t_inc / n * 1e3:.3f}")
