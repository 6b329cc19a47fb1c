"""Host-observed latency of one h-evaluation (lio_match round trip), C2 (diagnostics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import frontend as F  # noqa: E402
from lio_gpu import synth  # noqa: E402

scene, m, scans = synth.make_config("C2", n_scans=1)
sc = scans[0]
p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
tree = F.IkdTreeGPU(cell_size=1.0)
tree.Build(m)
hm = F.HShareModelGPU(tree)
hm.set_scan(sc.body)
hm(p24, True)
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(2000):
        hm(p24, False)
    t1 = time.perf_counter()
    for _ in range(500):
        hm(p24, True)
    t2 = time.perf_counter()
    print(f"{os.path.basename(os.environ.get('LIO_GPU_LIB', 'current'))} rep{rep} reuse_us={(t1 - t0) / 2000 * 1e6:6.1f} "
          f"redo_us={(t2 - t1) / 500 * 1e6:6.1f}", flush=True)
