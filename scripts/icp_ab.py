"""C4 loop-ICP timing (diagnostics): ms per alignment and per correspondence pass for the
1-iteration pair (0.3 m / 1.5 deg) and the multi-iteration pair (2.5 m / 4 deg).
Kernel choice by environment (LIO_ICP_KERNEL=tile for the round-1 tile kernel); LIO_ICP_ORDER=k times the
float order k (lio_icp_params.umeyama_float; default 2, the library default), -1 the opt-in double statistics."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import loop_closure as LC  # noqa: E402
from lio_gpu import synth  # noqa: E402

cell = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kern = os.environ.get("LIO_ICP_KERNEL", "tile")
order = int(os.environ.get("LIO_ICP_ORDER", "2"))  # -1: the opt-in double statistics
for disp in ((0.3, 1.5), (2.5, 4.0)):
    src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321, disp=disp)
    lc = LC.LoopClosure(LC.LoopClosureConfig(), cell_size=cell, umeyama_float=order)
    lc.setInputSource(src)
    lc.setInputTarget(dst)
    r = lc.align(keep_aligned=False)
    t0 = time.perf_counter()  # no timing events in the loop (they add marker packets between the kernels)
    for _ in range(reps):
        r = lc.align(keep_aligned=False)
    ms0 = (time.perf_counter() - t0) / reps * 1e3
    lc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = lc.align(keep_aligned=False)
    ms = (time.perf_counter() - t0) / reps * 1e3
    t = lc.timing()
    lc.set_timing(False)
    fs = lc.fidelity_stats() if order > 0 else {}
    print(f"order={order} {fs} kernel={kern} cell={cell} disp={disp} ms/align={ms0:.3f} timed_ms/align={ms:.3f} iters={r.iterations} "
          f"score={r.score:.6f} pass_ms={t['icp_ms'] / max(t['icp_launches'], 1):.4f} "
          f"passes/align={t['icp_launches'] / reps:.1f}", flush=True)
