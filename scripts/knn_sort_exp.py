"""Experiment: kNN kernel time vs query order (input voxel order vs Morton order)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402


def morton(p, res):
    v = np.clip(np.floor((p - p.min(0)) / res).astype(np.int64), 0, 1023)

    def spread(x):
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x

    return spread(v[:, 0]) | (spread(v[:, 1]) << 1) | (spread(v[:, 2]) << 2)


cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene, m, scans = synth.make_config(cfg, n_scans=1)
sc = scans[0]
p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build(m)
orders = {"input": np.arange(len(sc.body))}
for res in (0.25, 0.5, 1.0):
    orders[f"morton{res}"] = np.argsort(morton(sc.body, res), kind="stable")
for mode in ("lane", "group"):
    os.environ["LIO_KNN_MODE"] = mode
    for name, o in orders.items():
        hm = F.HShareModelGPU(tree)
        hm.set_scan(sc.body[o])
        hm.set_timing(True)
        for _ in range(20):
            s = hm(p24, True)
        t = hm.timing()
        print(f"{cfg} mode={mode:5s} order={name:10s} knn_avg_us={t['knn_ms'] / t['knn_launches'] * 1e3:7.1f} n_eff={int(s[27])}",
              flush=True)
        hm.close()
