"""kNN / h-model kernel timing and search statistics on the GPU box (diagnostics)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
cell = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
scene, m, scans = synth.make_config(cfg, n_scans=1)
sc = scans[0]
p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
tree = F.IkdTreeGPU(cell_size=cell)
tree.Build(m)
hm = F.HShareModelGPU(tree)
hm.set_scan(sc.body)
sums, s = hm.knn_stats(p24)
print(f"{cfg} cell={cell} n={len(sc.body)} n_eff={int(sums[27])} shell hist {np.bincount(s[:, 2], minlength=3).tolist()} "
      f"cells mean {s[:, 0].mean():.1f} points mean {s[:, 1].mean():.1f}", flush=True)
for rep in range(3):
    hm.reset_timing()
    hm.set_timing(True)
    for _ in range(50):
        hm(p24, True)
        hm(p24, False)
    t = hm.timing()
    hm.set_timing(False)
    print(f"rep{rep} redo_us={t['knn_ms'] / t['knn_launches'] * 1e3:7.1f} reuse_us={t['reuse_ms'] / t['reuse_launches'] * 1e3:6.1f}", flush=True)
