"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture bit-for-bit (it is pinned against
regressions).  GPU: the HIP path matches the fixtures (kNN ids, gates and
planes bit-exact; sums and IESKF within the north_star tolerances).
"""
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def _state(vec):
    keys = [("pos", 3), ("rot", 4), ("offset_R_L_I", 4), ("offset_T_L_I", 3), ("vel", 3), ("bg", 3), ("ba", 3),
            ("grav", 3)]
    out, o = {}, 0
    for k, n in keys:
        out[k] = np.asarray(vec[o:o + n], float)
        o += n
    return out


def test_oracle_reproduces_frontend_fixture(oracle):
    f = _load("frontend_small.npz")
    om = oracle.OracleMap(f["map"])
    np.testing.assert_array_equal(oracle.body_to_world(f["pose24"], f["body"]), f["world"])
    idx, d2 = om.knn(f["world"], 5, 5.0)
    np.testing.assert_array_equal(idx, f["knn_idx"])
    np.testing.assert_array_equal(d2, f["knn_d2"])
    n = len(f["body"])
    nn = np.full((n, 5), -1, np.int32)
    sel = np.zeros(n, np.uint8)
    planes = np.zeros((n, 4), np.float32)
    sums = oracle.h_share_model(om, f["body"], f["pose24"], True, nn, sel, planes)
    np.testing.assert_array_equal(nn, f["nn_idx"])
    np.testing.assert_array_equal(sel, f["sel"])
    np.testing.assert_array_equal(planes, f["planes"])
    np.testing.assert_array_equal(sums, f["sums"])
    sums = oracle.h_share_model(om, f["body"], f["pose24_b"], False, nn, sel, planes)
    np.testing.assert_array_equal(sel, f["sel_b"])
    np.testing.assert_array_equal(sums, f["sums_b"])
    x, P, stats, _ = oracle.ieskf_update(om, f["body"], _state(f["x0"]), f["P0"])
    np.testing.assert_array_equal(np.concatenate([x[k] for k in _state(f["x0"])]), f["x1"])
    np.testing.assert_array_equal(P, f["P1"])


def test_oracle_reproduces_esti_plane_fixture(oracle):
    f = _load("esti_plane.npz")
    for P5, o, ok in zip(f["pts"], f["out"], f["ok"]):
        got_ok, got = oracle.esti_plane(P5, 0.1)
        assert got_ok == bool(ok)
        np.testing.assert_array_equal(got, o)
    assert 0 < f["ok"].sum() < len(f["ok"])  # both branches of the flatness gate are covered


def test_oracle_reproduces_icp_fixture(oracle):
    f = _load("icp_small.npz")
    assert int(f["umeyama_order"]) == 2  # the default arithmetic: PCL's float Umeyama, Eigen 3.3 order
    r = oracle.icp_align(f["src"], f["dst"], want_aligned=True)
    np.testing.assert_array_equal(r["T"], f["T"])
    assert r["iterations"] == int(f["iterations"]) and r["state"] == int(f["state"])
    assert r["fitness"] == float(f["fitness"])
    np.testing.assert_array_equal(r["aligned"], f["aligned"])


@pytest.mark.gpu
def test_gpu_matches_frontend_fixture():
    from lio_gpu import frontend as F

    f = _load("frontend_small.npz")
    tree = F.IkdTreeGPU()
    tree.Build(f["map"])
    hm = F.HShareModelGPU(tree)
    hm.set_scan(f["body"])
    g = hm(f["pose24"], True)
    np.testing.assert_array_equal(hm.world(), f["world"])
    gi, gd = hm.nearest_points()
    np.testing.assert_array_equal(gi, f["nn_idx"])
    np.testing.assert_array_equal(gd, f["knn_d2"])
    gp, gs = hm.normvec()
    np.testing.assert_array_equal(gs, f["sel"])
    k = gs.astype(bool)
    np.testing.assert_array_equal(gp[k], f["planes"][k])
    np.testing.assert_allclose(g[:30], f["sums"][:30], rtol=1e-9, atol=1e-9)
    g2 = hm(f["pose24_b"], False)
    _, gs2 = hm.normvec()
    np.testing.assert_array_equal(gs2, f["sel_b"])
    np.testing.assert_allclose(g2[:30], f["sums_b"][:30], rtol=1e-9, atol=1e-9)
    kf = F.EsekfGPU(hm)
    x, P, st = kf.update_iterated_dyn_share_modified(_state(f["x0"]), f["P0"])
    x1 = _state(f["x1"])
    np.testing.assert_allclose(x["pos"], x1["pos"], atol=1e-5)
    np.testing.assert_allclose(x["rot"], x1["rot"], atol=1e-5)
    np.testing.assert_allclose(P, f["P1"], rtol=1e-5, atol=1e-10)
    assert st["h_evals"] == int(f["ieskf_stats"][0])


@pytest.mark.gpu
def test_gpu_matches_icp_fixture():
    from lio_gpu import loop_closure as LC

    f = _load("icp_small.npz")
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    lc.icpAlignment(f["src"], f["dst"])
    r = lc.last_result
    assert r.iterations == int(f["iterations"]) and r.state == int(f["state"])
    np.testing.assert_allclose(np.array(list(r.T), np.float32).reshape(4, 4), f["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, float(f["fitness"]), rtol=1e-5)
    np.testing.assert_allclose(lc.getFinalAlignedCloud(), f["aligned"], atol=1e-4)
