"""kNN kernel diagnostics on the GPU box: search statistics and a cell-size sweep."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
cells = [float(c) for c in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0.5", "0.75", "1.0", "1.5", "2.0", "3.0"])]
scene, m, scans = synth.make_config(cfg, n_scans=2)
sc = scans[0]
st = synth.initial_state(sc.pos_init, sc.rot_init)
p24 = synth.pose24(st)
for cell in cells:
    tree = F.IkdTreeGPU(cell_size=cell)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    sums, s = hm.knn_stats(p24)
    hm.set_timing(True)
    for _ in range(20):
        hm(p24, True)
    t = hm.timing()
    print(f"{cfg} cell={cell:.2f} grid={tree.grid()['dims'].tolist()} n_eff={int(sums[27])} "
          f"knn_avg_us={t['knn_ms'] / t['knn_launches'] * 1e3:.1f} | "
          f"cells mean {s[:, 0].mean():.1f} p99 {np.percentile(s[:, 0], 99):.0f} max {s[:, 0].max()} | "
          f"points mean {s[:, 1].mean():.1f} p99 {np.percentile(s[:, 1], 99):.0f} max {s[:, 1].max()} | "
          f"shell hist {np.bincount(s[:, 2], minlength=5).tolist()}", flush=True)
    hm.close()
    tree.close()
