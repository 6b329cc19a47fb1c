"""How much does the SO3 evaluation form matter?  (VERDICT r01 "What's weak" 2a)

FAST-LIO computes p_world = s.rot * (s.offset_R_L_I * p + t_LI) + pos with MTK::SO3 =
Eigen::Quaternion<double>, i.e. through QuaternionBase::_transformVector.  Round 1 used the
rotation matrix of the quaternion instead.  This script counts, on the synthetic C2 / C3 scans
(static maps of the configs' sizes; C3's map here is sampled, not grown), how many float world points,
5-NN id lists, and kNN-gate outcomes differ between the two forms:

    world_q = oracle (quaternion, the form now used by the oracle and the kernels)
    world_m = ((R0 b0 + R1 b1) + R2 b2) + t, the round-1 matrix form, replicated element-wise in numpy

Usage: python scripts/quat_vs_matrix.py [C2 C3]   (CPU only; a few minutes at C3)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
from lio_gpu import synth  # noqa: E402


def world_matrix(p, body):
    R, t, RLI, tLI = p[0:9], p[9:12], p[12:21], p[21:24]
    b = body.astype(np.float64)
    pi = [((RLI[3 * r] * b[:, 0] + RLI[3 * r + 1] * b[:, 1]) + RLI[3 * r + 2] * b[:, 2]) + tLI[r] for r in range(3)]
    w = [((R[3 * r] * pi[0] + R[3 * r + 1] * pi[1]) + R[3 * r + 2] * pi[2]) + t[r] for r in range(3)]
    return np.stack(w, axis=1).astype(np.float32)


def main(cfgs):
    out = {}
    for cfg in cfgs:
        scene, m, scans = synth.make_config(cfg, n_scans=3)
        om = O.OracleMap(m)
        acc = dict(points=0, world_diff=0, knn_list_diff=0, gate_diff=0)
        for sc in scans:
            # a pose off the ground truth, as in the first IESKF iteration, and a rotated one
            for st in (synth.initial_state(sc.pos_init, sc.rot_init), synth.initial_state(sc.pos_gt, sc.rot_gt)):
                p = synth.pose24(st)
                wq = O.body_to_world(p, sc.body)
                wm = world_matrix(p, sc.body)
                dif = np.any(wq != wm, axis=1)
                iq, dq = om.knn(wq, 5, 5.0)
                im, dm = om.knn(wm, 5, 5.0)
                gate_q = (iq[:, 4] >= 0) & (dq[:, 4] <= 5.0)
                gate_m = (im[:, 4] >= 0) & (dm[:, 4] <= 5.0)
                acc["points"] += len(sc.body)
                acc["world_diff"] += int(dif.sum())
                acc["knn_list_diff"] += int(np.any(iq != im, axis=1).sum())
                acc["gate_diff"] += int((gate_q != gate_m).sum())
        acc["world_diff_frac"] = acc["world_diff"] / acc["points"]
        acc["knn_list_diff_frac"] = acc["knn_list_diff"] / acc["points"]
        out[cfg] = acc
        print(cfg, json.dumps(acc), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:] or ["C2", "C3"])
