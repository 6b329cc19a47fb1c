"""C5 scan preprocessing host wall time per sweep: lio_scan_preprocess on 120k-point
KITTI-64 raw sweeps (Preprocess point_filter_num 4, blind 2, UndistortPcl, downSizeFilterSurf 0.5) into a
ctx, median / p90 over `reps` calls cycling through 6 sweeps.  A/B: LIO_PREP_UPLOAD=full (the whole sweep
uploaded from pageable memory, selected on the device) and LIO_GPU_LIB=<older build>.  Also times the same
calls from a pinned copy of the sweeps (torch pin_memory), the zero-copy receive buffer a driver can use.

usage: python scripts/prep_timing.py [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
scene = synth.make_scene(4000.0, 1234)
sweeps = [synth.make_raw_scan(scene, 120_000, seed=30 + k) for k in range(6)]
m = synth.sample_surface(scene, 400_000, 1234)
tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
tree.Build(m)
hm = F.HShareModelGPU(tree)
ends = [F.pose_from_pose24(e) for _, _, e in sweeps]


def run(raws):
    t = []
    for k in range(reps + 5):
        j = k % len(sweeps)
        t0 = time.perf_counter()
        n = hm.preprocess_scan(raws[j], sweeps[j][1], ends[j], point_filter_num=4, blind=2.0, filter_size_surf=0.5)
        if k >= 5:
            t.append((time.perf_counter() - t0) * 1e3)
    t = np.array(t)
    return n, float(np.median(t)), float(np.percentile(t, 90)), float(t.mean())


tag = f"lib={os.environ.get('LIO_GPU_LIB', 'HEAD')} upload={os.environ.get('LIO_PREP_UPLOAD', 'staged')}"
n, p50, p90, mean = run([s[0] for s in sweeps])
print(f"{tag} pageable: n_down {n} ms/sweep p50 {p50:.4f} p90 {p90:.4f} mean {mean:.4f}", flush=True)
try:
    import torch

    pinned = [torch.from_numpy(s[0]).pin_memory().numpy() for s in sweeps]
    n, p50, p90, mean = run(pinned)
    print(f"{tag} pinned:   n_down {n} ms/sweep p50 {p50:.4f} p90 {p90:.4f} mean {mean:.4f}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"pinned leg skipped: {e}", flush=True)
