"""The first map_incremental call's set-up: per-call host times of the first few
map_incremental calls on the C3 map (5 M points) after an IESKF update each.  Run it with and without
HIP_ENABLE_DEFERRED_LOADING=0 (code objects loaded at start-up instead of at each kernel's first launch)
to split buffer set-up from kernel loading."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
import numpy as np  # noqa: E402

from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

mp, L, sp, kind = synth.CONFIGS["C3"]
scene = synth.make_scene(L, 1234)
m = synth.sample_surface(scene, mp, 1234)
tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
t0 = time.perf_counter()
tree.Build(m)
build_ms = (time.perf_counter() - t0) * 1e3
hm = F.HShareModelGPU(tree)
kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
times = []
for k in range(5):
    x = -0.15 * L + 1.85 + k * 3.7
    sc = synth.make_scan(scene, sp, kind, pos_gt=[x, 0.6 * np.sin(0.7 * k + 0.3), 0.0], yaw_gt=0.0, seed=5099 + k)
    hm.set_scan(sc.body)
    xg, _, _ = kf.update_iterated_dyn_share_modified(synth.initial_state(sc.pos_init, sc.rot_init), synth.initial_cov())
    t0 = time.perf_counter()
    hm.map_incremental(synth.pose24(xg), 0.5)
    times.append((time.perf_counter() - t0) * 1e3)
print(f"deferred_loading={os.environ.get('HIP_ENABLE_DEFERRED_LOADING', 'default')} build {build_ms:.1f} ms; "
      f"map_incremental ms per call: " + " ".join(f"{t:.3f}" for t in times), flush=True)
