"""ICP (C4) alignment time vs target grid cell size (diagnostics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import loop_closure as LC  # noqa: E402
from lio_gpu import synth  # noqa: E402

src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321)
cells = [float(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1.0", "1.5", "2.0", "3.0", "4.0"])]
for cell in cells:
    lc = LC.LoopClosure(LC.LoopClosureConfig(), cell_size=cell)
    lc.setInputSource(src)
    lc.setInputTarget(dst)
    r = lc.align(keep_aligned=False)
    lc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(5):
        r = lc.align(keep_aligned=False)
    ms = (time.perf_counter() - t0) / 5 * 1e3
    t = lc.timing()
    print(f"cell={cell:.2f} ms/align={ms:.3f} iters={r.iterations} score={r.score:.6f} "
          f"kernel_ms/pass={t['icp_ms'] / max(t['icp_launches'], 1):.4f} passes/align={t['icp_launches'] / 5:.1f}",
          flush=True)
