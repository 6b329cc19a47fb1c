"""Spread of PCL's float ICP result over Eigen-plausible summation orders.

pcl::umeyama's float sums have no single defined order: Eigen 3.3 sums the mean rows sequentially but
blocks sigma's depth by an L1-size-dependent kc (lio_oracle.cpp UmeyamaOrder).  This runs the oracle's ICP
(PCL 1.10 criteria, kd-tree 1-NN) on the C4 pairs at full size with every order and with the double
statistics, and prints the max |dT| between each pair of modes.

    python scripts/umeyama_spread.py [n_points] [threads]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402
from lio_gpu import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
    thr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for name, disp in (("A", (0.3, 1.5)), ("B", (2.5, 4.0))):
        src, dst, _ = synth.make_icp_pair(n_points=n, seed=4321, disp=disp)
        res = {}
        for order in [0] + sorted(O.UMEYAMA_ORDERS):
            p = O.default_icp_params()
            p.umeyama_float = order
            t0 = time.time()
            res[order] = O.icp_align(src, dst, params=p, threads=thr)
            r = res[order]
            print(f"pair {name} order {order} ({O.UMEYAMA_ORDERS.get(order, 'double statistics')}): iters "
                  f"{r['iterations']} state {r['state']} fitness {r['fitness']:.9g} ({time.time() - t0:.1f} s)",
                  flush=True)
        ks = sorted(res)
        print(f"pair {name}: max |dT| between modes (rows / cols: order; 0 = double statistics)")
        print("      " + " ".join(f"{k:>9d}" for k in ks))
        for a in ks:
            row = [float(np.abs(res[a]["T"] - res[b]["T"]).max()) for b in ks]
            print(f"{a:>5d} " + " ".join(f"{v:9.3g}" for v in row))
        fl = [k for k in ks if k > 0]
        spread = max(float(np.abs(res[a]["T"] - res[b]["T"]).max()) for a in fl for b in fl)
        plaus = [1, 2, 3]
        spread_p = max(float(np.abs(res[a]["T"] - res[b]["T"]).max()) for a in plaus for b in plaus)
        dd = max(float(np.abs(res[0]["T"] - res[k]["T"]).max()) for k in fl)
        print(f"pair {name}: spread over float orders {spread:.3g} (Eigen 3.3 orders 1-3: {spread_p:.3g}); "
              f"double statistics to the farthest float order {dd:.3g}", flush=True)


if __name__ == "__main__":
    main()
