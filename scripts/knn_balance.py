"""Per-query / per-wave work distribution of the front-end near kNN pass (diagnostics)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene, m, scans = synth.make_config(cfg, n_scans=1)
sc = scans[0]
p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
tree = F.IkdTreeGPU()
tree.Build(m)
hm = F.HShareModelGPU(tree)
hm.set_scan(sc.body)
sums, s = hm.knn_stats(p24)
pts = s[:, 1].astype(np.int64)
print("points/query pct 50/90/99/99.9/max:", np.percentile(pts, [50, 90, 99, 99.9]).round(1), pts.max())
w = pts[: len(pts) // 8 * 8].reshape(-1, 8)  # 8 queries per wave
wm = w.max(1)
print("per-wave max points pct 50/90/99/max:", np.percentile(wm, [50, 90, 99]).round(1), wm.max())
print("per-wave sum points pct 50/90/99/max:", np.percentile(w.sum(1), [50, 90, 99]).round(1), w.sum(1).max())
# own-cell sizes of the map grid
far = (s[:, 2] == 2).astype(np.int64)
fb = far[: len(far) // 64 * 64].reshape(-1, 64).sum(1)
print("far queries:", int(far.sum()), "per 64-query block: max", int(fb.max()), "blocks with >0:", int((fb > 0).sum()),
      "hist", np.bincount(fb)[:12].tolist())
