"""Full-size parity for the BASELINE.json configurations the other GPU tests cover only in part
(VERDICT r01 "What's missing" #4):

* C3 — a 5 M-point map GROWN through 20 map_incremental calls (the bench's growth drive), the
  oracle replaying every insert with the same kNN / final poses: map content bit-exact after the
  drive, then one kNN evaluation (ids bit-exact) and one full IESKF update (pose within 1e-5) on
  the grown map.
* C5 — three raw 120 k-point KITTI-64 sweeps through the whole front end on a 10 M-point map:
  Preprocess + UndistortPcl + downSizeFilterSurf (bit-exact), the IESKF update (pose within 1e-5 of
  the oracle's update of its OWN preprocess output), map_incremental given the same poses (map
  bit-exact).  The stream with its loop leg: tests/test_gpu_pipeline.py.
* C4 — the sharded loop ICP with 4 emulated ranks at 500 k points (2.5 m / 4 deg offset, 9
  iterations): every rank's transform bit-identical to the 1-rank alignment.

Each test generates its inputs once (synth caches the full-size maps per process) and runs in
about a minute on the GPU box.
"""
import math
import threading

import numpy as np
import pytest

from lio_gpu import frontend as F
from lio_gpu import loop_closure as LC
from lio_gpu import synth

pytestmark = pytest.mark.gpu


def _same_map(tree, om):
    gx, ga = tree.by_id()
    ox, oa = om.by_id()
    assert gx.shape == ox.shape
    np.testing.assert_array_equal(ga, oa)
    np.testing.assert_array_equal(gx, ox)
    assert tree.size() == om.size()


def _identity_pose():
    p24 = np.zeros(24)
    p24[0:9] = np.eye(3).ravel()
    p24[12:21] = np.eye(3).ravel()
    return p24


@pytest.mark.timeout(600)
def test_c3_map_grown_by_map_incremental(oracle):
    mp, L, sp, kind = synth.CONFIGS["C3"]
    scene = synth.make_scene(L, 1234)
    m = synth.sample_surface(scene, mp, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(m)
    om = oracle.OracleDynMap(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
    P0 = synth.initial_cov()
    offered = 0
    for k in range(20):  # bench.py's growth drive (filter_size_map = 0.5, kitti.launch:10)
        x = -0.15 * L + 1.85 + k * 3.7
        s = synth.make_scan(scene, sp, kind, pos_gt=[x, 0.6 * math.sin(0.7 * k + 0.3), 0.0],
                            yaw_gt=0.05 * math.sin(0.3 * k + 0.2), seed=5099 + k)
        hm.set_scan(s.body)
        xg, _, _ = kf.update_iterated_dyn_share_modified(synth.initial_state(s.pos_init, s.rot_init), P0)
        p_knn, p_fin = hm.last_knn_pose24(), synth.pose24(xg)
        sg = hm.map_incremental(p_fin, 0.5)
        assert sg == om.map_incremental(s.body, p_knn, p_fin, 0.5, 0.5)
        offered += sg["n_to_add"] + sg["n_no_downsample"]
    assert offered > 100_000 and tree.num_ids() > mp
    _same_map(tree, om)
    # a scan against the grown map: kNN ids bit-exact, then a full IESKF update
    sc = synth.make_scan(scene, sp, kind, pos_gt=[-0.15 * L + 20.0, 0.3, 0.0], yaw_gt=0.02, seed=6100)
    tv = om.tree()
    hm.set_scan(sc.body)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    p24 = synth.pose24(st)
    g = hm(p24, True)
    n = len(sc.body)
    nn = np.full((n, 5), -1, np.int32)
    sel = np.zeros(n, np.uint8)
    planes = np.zeros((n, 4), np.float32)
    o = oracle.h_share_model(tv, sc.body, p24, True, nn, sel, planes)
    gi, _ = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    assert int(g[27]) == int(o[27]) > 1000
    np.testing.assert_allclose(g[:27], o[:27], rtol=1e-9, atol=1e-9)
    xg, Pg, sg = kf.update_iterated_dyn_share_modified(st, P0)
    xo, Po, so, _ = oracle.ieskf_update(tv, sc.body, st, P0)
    assert sg["h_evals"] == int(so[0])
    np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
    np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
    np.testing.assert_allclose(Pg, Po, rtol=1e-5, atol=1e-12)
    hm.close()


@pytest.mark.timeout(600)
def test_c5_raw_scan_pipeline_three_scans(oracle):
    mp, L, sp, kind = synth.CONFIGS["C5"]
    scene = synth.make_scene(L, 1234)
    m = synth.sample_surface(scene, mp, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(m)
    om = oracle.OracleDynMap(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
    P0 = synth.initial_cov()
    delta = synth.rotvec_to_quat(np.deg2rad([0.5, -0.4, 1.0]))
    for k in range(3):  # bench.py --pipeline's drive
        x0 = -0.15 * L + 0.9 + k * 3.7
        raw, poses, end24 = synth.make_raw_scan(scene, sp, "kitti64", seed=777 + k,
                                                origin=(x0, 0.4 * math.sin(0.5 * k), 0.0), yaw0=0.04 * math.sin(0.2 * k))
        n_down = hm.preprocess_scan(raw, poses, F.pose_from_pose24(end24), point_filter_num=4, blind=2.0,
                                    filter_size_surf=0.5, time_field=4)
        o = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.5)
        assert n_down == len(o) > 1000
        hm(_identity_pose(), True)
        # feats_down_body as the device holds it (identity pose: world == body): the oracle's own, bit for bit
        np.testing.assert_array_equal(hm.world(), o[:, :3])
        body = np.ascontiguousarray(o[:, :3])
        R_e = end24[0:9].reshape(3, 3)
        q_e = synth.rotvec_to_quat([0.0, 0.0, float(np.arctan2(R_e[1, 0], R_e[0, 0]))])
        st0 = synth.initial_state(end24[9:12] + np.array([0.10, -0.08, 0.05]), synth.quat_mul(q_e, delta))
        xg, Pg, sg = kf.update_iterated_dyn_share_modified(st0, P0)
        xo, Po, so, _ = oracle.ieskf_update(om.tree(), body, st0, P0)
        assert sg["h_evals"] == int(so[0]) and sg["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        assert np.linalg.norm(xg["pos"] - end24[9:12]) < 0.2
        p_knn, p_fin = hm.last_knn_pose24(), synth.pose24(xg)
        assert hm.map_incremental(p_fin, 0.5) == om.map_incremental(body, p_knn, p_fin, 0.5, 0.5)
        _same_map(tree, om)
    hm.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,disp", [(4, (2.5, 4.0)), (2, (0.3, 1.5)), (8, (2.5, 4.0))])
def test_icp_c4_emulated_ranks_bit_identical(oracle, world, disp):
    """BASELINE.json configs[3]'s layout: the source sharded over `world` ranks (threads, one LoopClosure
    each, in-process host all-gathers), target replicated, in the DEFAULT mode (PCL's float Umeyama, Eigen 3.3
    order) with the float chains split over the ranks' windows (round 6: block sums, event lists and depth blocks
    exchanged; each rank holds only its shard): every rank's transform equals the one-rank transform bit for
    bit, and that transform is within 1e-5 of the oracle's float order 2."""
    src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321, disp=disp)
    bar = threading.Barrier(world)
    slots = [None] * world
    results = [None] * world
    from lio_gpu import _capi

    def make_cb(rank):
        def cb(send_p, n, recv_p, user):
            slots[rank] = np.ctypeslib.as_array(send_p, shape=(n,)).copy()
            bar.wait()
            np.ctypeslib.as_array(recv_p, shape=(n * world,))[:] = np.concatenate(slots)
            bar.wait()
            return 0

        return _capi.ALLGATHER_FN(cb)

    cbs = [make_cb(r) for r in range(world)]
    lcs = [LC.LoopClosure(LC.LoopClosureConfig()) for _ in range(world)]

    def run(rank):
        lcs[rank].set_shard(rank, world, cbs[rank])
        lcs[rank].setInputSource(src)
        lcs[rank].setInputTarget(dst)
        results[rank] = lcs[rank].align(keep_aligned=False)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(timeout=300) for t in th]
    single = LC.LoopClosure(LC.LoopClosureConfig())
    single.setInputSource(src)
    single.setInputTarget(dst)
    r1 = single.align(keep_aligned=False)
    assert r1.iterations >= (5 if disp[0] > 1 else 1)
    T1 = np.array(list(r1.T), np.float32)
    for r in results:
        assert r is not None
        np.testing.assert_array_equal(np.array(list(r.T), np.float32), T1)
        assert r.score == r1.score and r.iterations == r1.iterations
    # the re-passes and re-exchanges recover on the sharded path as on one rank: no serial fallback
    if single.fidelity_stats()["serial"] == 0:
        assert all(lc.fidelity_stats()["serial"] == 0 for lc in lcs), [lc.fidelity_stats() for lc in lcs]
    o = oracle.icp_align(src, dst)  # float order 2 (oracle default)
    assert r1.iterations == o["iterations"] and r1.state == o["state"]
    np.testing.assert_allclose(T1.reshape(4, 4), o["T"], atol=1e-5)
