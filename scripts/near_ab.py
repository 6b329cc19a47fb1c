#!/usr/bin/env python3
"""Near-pass A/B between library builds (LIO_GPU_LIB): per-kernel event timing of the unseeded and the
seeded near pass at C3 (static 5 M map), plus the search statistics.  Diagnostics only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
scene, m, scans = synth.make_config(cfg, n_scans=1)
sc = scans[0]
p0 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
p1 = synth.pose24(synth.initial_state(sc.pos_gt, sc.rot_gt))
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build(m)
hm = F.HShareModelGPU(tree)
hm.set_scan(sc.body)
sums, s = hm.knn_stats(p0)
lib = os.path.basename(os.path.dirname(os.environ.get("LIO_GPU_LIB", "current/x")))


def phase(seeded):
    hm.reset_timing()
    for _ in range(5):  # warm-up
        hm.set_scan(sc.body)
        hm(p0, True)
        if seeded:
            hm(p1, True)
    hm.reset_timing()
    hm.set_timing(True)
    for _ in range(reps):
        hm.set_scan(sc.body)
        hm(p0, True)
        if seeded:
            hm(p1, True)
    hm.set_timing(False)
    return hm.timing()


a = phase(False)
b = phase(True)
un = a["near_ms"] / a["near_launches"] * 1e3
se = (b["near_ms"] * 1e3 - un * reps) / reps
print(f"{cfg} lib={lib} points/query {s[:, 1].mean():.1f} cells/query {s[:, 0].mean():.1f} | near unseeded {un:.2f} us "
      f"seeded {se:.2f} us | far {a['far_ms'] / a['far_launches'] * 1e3:.2f} us plane {a['plane_ms'] / a['plane_launches'] * 1e3:.2f} us",
      flush=True)
