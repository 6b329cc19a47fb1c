"""Where the whole icpAlignment's set-up goes: setInputTarget (upload + target grid),
setInputSource + the first align's preparation (upload + source binning + tiles), the alignment itself —
host wall times on a warm handle, C4 pair B (500 k vs 500 k), median of 7."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import loop_closure as LC  # noqa: E402
from lio_gpu import synth  # noqa: E402

order = int(os.environ.get("LIO_ICP_ORDER", "2"))  # -1: the opt-in double statistics
src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321, disp=(2.5, 4.0))
lc = LC.LoopClosure(LC.LoopClosureConfig(), umeyama_float=order)
lc.setInputSource(src)
lc.setInputTarget(dst)
lc.align(keep_aligned=False)
rows = []
for _ in range(7):
    t0 = time.perf_counter()
    lc.setInputTarget(dst)
    t1 = time.perf_counter()
    lc.setInputSource(src)
    t2 = time.perf_counter()
    lc.align(keep_aligned=False)  # includes the source preparation (deferred to the first align)
    t3 = time.perf_counter()
    lc.align(keep_aligned=False)  # warm: the alignment alone
    t4 = time.perf_counter()
    rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3))
m = np.median(np.array(rows), axis=0)
print(f"order={order} setInputTarget {m[0]:.3f} ms | setInputSource {m[1]:.3f} ms | first align (prep + align) "
      f"{m[2]:.3f} ms | align alone {m[3]:.3f} ms | full = {m[0] + m[1] + m[2]:.3f} ms", flush=True)
