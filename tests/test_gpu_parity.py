"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle.

Bars (BASELINE.json north_star): kNN ids bit-exact; world points, planes,
gates bit-exact (same float op order, -ffp-contract=off on both sides);
H^T H / H^T h within 1e-9 relative (double sums in a different order);
IESKF pose within 1e-5; ICP transform within 1e-5.
"""
import threading

import numpy as np
import pytest

from lio_gpu import frontend as F
from lio_gpu import loop_closure as LC
from lio_gpu import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1():
    scene, m, scans = synth.make_config("C1", n_scans=2)
    return scene, m, scans


def _oracle_eval(oracle, om, body, p24, nn=None, sel=None, planes=None, redo=True):
    n = len(body)
    nn = np.full((n, 5), -1, np.int32) if nn is None else nn
    sel = np.zeros(n, np.uint8) if sel is None else sel
    planes = np.zeros((n, 4), np.float32) if planes is None else planes
    sums = oracle.h_share_model(om, body, p24, redo, nn, sel, planes)
    return sums, nn, sel, planes


def _check_sums(g, o):
    assert int(g[27]) == int(o[27])
    np.testing.assert_allclose(g[:27], o[:27], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(g[28:30], o[28:30], rtol=1e-9, atol=1e-9)


def test_map_roundtrip(c1):
    _, m, _ = c1
    t = F.IkdTreeGPU(cell_size=1.0)
    t.Build(m)
    assert t.size() == len(m)
    np.testing.assert_array_equal(t.points(), m)
    g = t.grid()
    assert g["cell"] == 1.0 and np.all(g["dims"] > 2)


@pytest.mark.parametrize("cell", [1.0, 0.6, 2.3])
def test_h_model_bit_exact_c1(oracle, c1, cell):
    _, m, scans = c1
    sc = scans[0]
    tree = F.IkdTreeGPU(cell_size=cell)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    p24 = synth.pose24(st)
    g = hm(p24, converge=True)
    om = oracle.OracleMap(m)
    o, nn, sel, planes = _oracle_eval(oracle, om, sc.body, p24)
    # world points
    np.testing.assert_array_equal(hm.world(), oracle.body_to_world(p24, sc.body))
    # kNN ids + sq-distances bit-exact
    gi, gd = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    oi, od = om.knn(oracle.body_to_world(p24, sc.body), 5, 5.0)
    np.testing.assert_array_equal(gd, od)
    # gates, planes, pd2 bit-exact
    gp, gs = hm.normvec()
    np.testing.assert_array_equal(gs, sel)
    k = sel.astype(bool)
    np.testing.assert_array_equal(gp[k], planes[k])
    _check_sums(g, o)


def test_reuse_path_matches_oracle(oracle, c1):
    _, m, scans = c1
    sc = scans[0]
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    om = oracle.OracleMap(m)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    p24 = synth.pose24(st)
    hm(p24, True)
    _, nn, sel, planes = _oracle_eval(oracle, om, sc.body, p24)
    # second evaluation at a moved pose without kNN (ekfom_data.converge == false)
    st2 = dict(st)
    st2["pos"] = st["pos"] + np.array([0.02, -0.01, 0.005])
    st2["rot"] = synth.quat_mul(st["rot"], synth.rotvec_to_quat([0.001, -0.002, 0.003]))
    p2 = synth.pose24(st2)
    g = hm(p2, converge=False)
    o, nn, sel, planes = _oracle_eval(oracle, om, sc.body, p2, nn, sel, planes, redo=False)
    gp, gs = hm.normvec()
    np.testing.assert_array_equal(gs, sel)
    k = sel.astype(bool)
    np.testing.assert_array_equal(gp[k, 3], planes[k, 3])
    _check_sums(g, o)


def test_ieskf_update_matches_oracle(oracle, c1):
    _, m, scans = c1
    om = oracle.OracleMap(m)
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm)
    for sc in scans:
        hm.set_scan(sc.body)
        st = synth.initial_state(sc.pos_init, sc.rot_init)
        P0 = synth.initial_cov()
        xg, Pg, sg = kf.update_iterated_dyn_share_modified(st, P0)
        xo, Po, so, _ = oracle.ieskf_update(om, sc.body, st, P0)
        assert sg["h_evals"] == int(so[0]) and sg["knn_calls"] == int(so[1])
        assert sg["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        np.testing.assert_allclose(Pg, Po, rtol=1e-5, atol=1e-10)
        assert np.linalg.norm(xg["pos"] - sc.pos_gt) < 0.2 * np.linalg.norm(sc.pos_init - sc.pos_gt)


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_ieskf_update_full_size(oracle, cfg):
    """Whole update_iterated_dyn_share_modified at BASELINE sizes: same evaluation / kNN counts and
    effective points as the oracle, state and covariance within the north_star tolerance."""
    _, m, scans = synth.make_config(cfg, n_scans=2)
    om = oracle.OracleMap(m)
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm)
    for sc in scans:
        hm.set_scan(sc.body)
        st = synth.initial_state(sc.pos_init, sc.rot_init)
        P0 = synth.initial_cov()
        xg, Pg, sg = kf.update_iterated_dyn_share_modified(st, P0)
        xo, Po, so, _ = oracle.ieskf_update(om, sc.body, st, P0)
        assert sg["h_evals"] == int(so[0]) and sg["knn_calls"] == int(so[1])
        assert sg["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        np.testing.assert_allclose(Pg, Po, rtol=1e-5, atol=1e-10)


def test_queries_just_outside_the_grid(oracle):
    """Scan points whose cell lies outside the map grid but within the kNN range of its faces:
    the near pass hands them to the far pass, which must search the whole box (the near pass
    scanned nothing for them). Nearest_Points bit-exact against the oracle."""
    rng = np.random.default_rng(8)
    m = rng.uniform(0.0, 10.0, (60000, 3)).astype(np.float32)
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    om = oracle.OracleMap(m)
    q = rng.uniform(0.0, 10.0, (6000, 3))
    axis = rng.integers(0, 3, len(q))
    side = rng.integers(0, 2, len(q))
    off = rng.uniform(0.05, 2.5, len(q))
    q[np.arange(len(q)), axis] = np.where(side == 1, 10.0 + off, -off)
    body = (q - synth.T_LI).astype(np.float32)  # identity pose: world = body + t_LI
    hm = F.HShareModelGPU(tree)
    hm.set_scan(body)
    p24 = np.zeros(24)
    p24[0:9] = np.eye(3).ravel()
    p24[12:21] = np.eye(3).ravel()
    p24[21:24] = synth.T_LI
    g = hm(p24, True)
    o, nn, sel, _ = _oracle_eval(oracle, om, body, p24)
    gi, _ = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    np.testing.assert_array_equal(hm.normvec()[1], sel)
    _check_sums(g, o)
    assert (gi[:, 4] >= 0).sum() > len(q) // 2 and (gi[:, 0] < 0).sum() > 0  # both kinds present


def test_edge_cases(oracle):
    rng = np.random.default_rng(5)
    # tiny map with duplicates (ties broken by id) and sparse areas (< 5 neighbours)
    m = rng.uniform(-4, 4, (400, 3)).astype(np.float32)
    m[:, 2] *= 0.05
    m = np.concatenate([m, m[:40], np.array([[30, 30, 0], [30.5, 30, 0]], np.float32)])
    tree = F.IkdTreeGPU(cell_size=0.7)
    tree.Build(m)
    om = oracle.OracleMap(m)
    body = np.concatenate([
        rng.uniform(-4, 4, (300, 3)),
        m[:40] - synth.T_LI,             # exactly on duplicated map points
        [[30, 30.2, 0], [500, 0, 0], [-1e4, 3, 2]],  # sparse / far outside the grid
    ]).astype(np.float32)
    body[:300, 2] *= 0.05
    hm = F.HShareModelGPU(tree)
    hm.set_scan(body)
    p24 = np.concatenate([np.eye(3).ravel(), np.zeros(3), np.eye(3).ravel(), synth.T_LI])
    g = hm(p24, True)
    o, nn, sel, planes = _oracle_eval(oracle, om, body, p24)
    gi, gd = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    assert (gi[-2:] == -1).all()  # nothing within sqrt(5) m
    gp, gs = hm.normvec()
    np.testing.assert_array_equal(gs, sel)
    _check_sums(g, o)
    # empty scan
    hm.set_scan(np.zeros((0, 3), np.float32))
    assert np.all(hm(p24, True) == 0)


def test_no_effective_points_and_small_dof_branch(oracle):
    # planar patch: only a handful of scan points land on it -> dof < 23 branch
    rng = np.random.default_rng(9)
    m = np.stack([rng.uniform(0, 10, 4000), rng.uniform(0, 10, 4000), rng.normal(0, 0.005, 4000)], 1).astype(np.float32)
    m[:, 2] += 3.0
    tree = F.IkdTreeGPU()
    tree.Build(m)
    om = oracle.OracleMap(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm)
    body_on = np.stack([rng.uniform(2, 8, 12), rng.uniform(2, 8, 12), np.full(12, 3.0)], 1) - synth.T_LI
    body_off = rng.uniform(50, 60, (100, 3))
    for body in (body_on.astype(np.float32), np.concatenate([body_on, body_off]).astype(np.float32),
                 body_off.astype(np.float32)):
        hm.set_scan(body)
        st = synth.initial_state([0.01, -0.02, 0.03], synth.rotvec_to_quat([0.002, 0, -0.001]))
        P0 = synth.initial_cov()
        xg, Pg, sg = kf.update_iterated_dyn_share_modified(st, P0)
        xo, Po, so, _ = oracle.ieskf_update(om, body, st, P0)
        assert sg["h_evals"] == int(so[0]) and sg["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-6)
        np.testing.assert_allclose(Pg, Po, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("cfg", ["C2", "C3", "C5"])
def test_knn_full_size(oracle, cfg):
    """BASELINE.json's full sizes (C2 65k/1M, C3 131k/5M, C5 120k/10M): Nearest_Points ids and
    point_selected_surf bit-exact, H^T H / H^T h sums within the double-order tolerance."""
    scene, m, scans = synth.make_config(cfg, n_scans=1)
    sc = scans[0]
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    p24 = synth.pose24(st)
    g = hm(p24, True)
    om = oracle.OracleMap(m)
    o, nn, sel, planes = _oracle_eval(oracle, om, sc.body, p24)
    gi, _ = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    gp, gs = hm.normvec()
    np.testing.assert_array_equal(gs, sel)
    _check_sums(g, o)


# ----------------------------------------------------------------------------- ICP
@pytest.fixture(scope="module")
def icp_small():
    return synth.make_icp_pair(n_points=30000, seed=21)


def _T(res):
    return np.array(list(res.T), np.float32).reshape(4, 4)


def test_icp_matches_oracle(oracle, icp_small):
    src, dst, Tgt = icp_small
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    out = lc.icpAlignment(src, dst)
    r = lc.last_result
    o = oracle.icp_align(src, dst, want_aligned=True)
    assert r.iterations == o["iterations"] and r.state == o["state"]
    np.testing.assert_allclose(_T(r), o["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, o["fitness"], rtol=1e-5)
    assert out.is_valid_ == o["is_valid"]
    np.testing.assert_allclose(lc.getFinalAlignedCloud(), o["aligned"], atol=1e-4)


def test_icp_sharded_two_handles_bit_identical(icp_small):
    """Two ranks emulated in one process (threads + in-process all-gather)."""
    src, dst, _ = icp_small
    world = 2
    lock = threading.Barrier(world)
    slots = [None] * world
    results = [None] * world

    def make_cb(rank):
        import ctypes as C

        from lio_gpu import _capi

        def cb(send_p, n, recv_p, user):
            slots[rank] = np.ctypeslib.as_array(send_p, shape=(n,)).copy()
            lock.wait()
            recv = np.ctypeslib.as_array(recv_p, shape=(n * world,))
            recv[:] = np.concatenate(slots)
            lock.wait()
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
    for r in results:
        assert r is not None
        np.testing.assert_array_equal(_T(r), _T(r1))
        assert r.score == r1.score and r.iterations == r1.iterations


def test_icp_c4_full_size_matches_oracle(oracle):
    src, dst, Tgt = synth.make_icp_pair(n_points=500_000, seed=4321)
    assert len(src) == 500_000 and len(dst) == 500_000
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    out = lc.icpAlignment(src, dst)
    r = lc.last_result
    o = oracle.icp_align(src, dst)
    assert r.is_converged and r.iterations == o["iterations"] and r.state == o["state"]
    np.testing.assert_allclose(_T(r), o["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, o["fitness"], rtol=1e-5)
    # size-independent property: the accepted step brought the clouds together
    assert r.score < r.last_mse
    assert out.score_ < 1.5 and out.is_valid_


def test_bind_scan_device_matches_copy(c1):
    """lio_scan_bind_device (caller-owned device scan, no copy) == lio_scan_set."""
    import torch

    _, m, scans = c1
    sc = scans[0]
    tree = F.IkdTreeGPU()
    tree.Build(m)
    p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
    h1 = F.HShareModelGPU(tree)
    h1.set_scan(sc.body)
    s1 = h1(p24, True)
    d = torch.from_numpy(sc.body).to("cuda:0")
    torch.cuda.synchronize()
    h2 = F.HShareModelGPU(tree)
    h2.bind_scan_device(d.data_ptr(), len(sc.body))
    s2 = h2(p24, True)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(h1.nearest_points()[0], h2.nearest_points()[0])
    np.testing.assert_array_equal(h1(p24, False), h2(p24, False))


@pytest.mark.parametrize("shift", [0.02, 0.3, 3.0])
def test_seeded_second_knn_bit_exact(oracle, c1, shift):
    """A later kNN evaluation of the same scan (map unchanged) starts from the triangle bound
    sqrt(previous d5) + displacement (group_knn_seeded): still the oracle's lists, bit-exact,
    for a small, a medium and a large pose change between the evaluations."""
    _, m, scans = c1
    sc = scans[0]
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    hm(synth.pose24(st), converge=True)  # first evaluation: unseeded
    st2 = dict(st)
    st2["pos"] = np.asarray(st["pos"]) + np.array([shift, -0.5 * shift, 0.25 * shift])
    p24 = synth.pose24(st2)
    g = hm(p24, converge=True)  # seeded by the first evaluation's lists
    om = oracle.OracleMap(m)
    o, nn, sel, planes = _oracle_eval(oracle, om, sc.body, p24)
    gi, gd = hm.nearest_points()
    np.testing.assert_array_equal(gi, nn)
    oi, od = om.knn(oracle.body_to_world(p24, sc.body), 5, 5.0)
    np.testing.assert_array_equal(gd, od)
    _check_sums(g, o)


@pytest.mark.parametrize("scale", [0.05, 0.5])
def test_seeded_guard_whole_box(oracle, scale):
    """The seeded pass's guard: a bound shrunk below the true 5th distance (lio_ctx_set_seed_scale)
    leaves lists that are not full; they are reset and the far pass searches the whole box, 3x3x3
    block included — the lists stay bit-exact."""
    scene, m, scans = synth.make_config("C1", n_scans=1)
    sc = scans[0]
    om = oracle.OracleMap(m)
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_seed_scale(scale)
    hm.set_scan(sc.body)
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    hm(synth.pose24(st), converge=True)
    for shift in (0.02, 0.3):
        st2 = dict(st)
        st2["pos"] = np.asarray(st["pos"]) + np.array([shift, -0.5 * shift, 0.25 * shift])
        p24 = synth.pose24(st2)
        hm(p24, converge=True)
        gi, gd = hm.nearest_points()
        oi, od = om.knn(oracle.body_to_world(p24, sc.body), 5, 5.0)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gd, od)
    hm.close()


@pytest.mark.parametrize("epsi,max_iter", [(0.001, 3), (0.05, 3), (1.0, 3), (1.0, 5), (0.001, 1), (0.02, 6)])
def test_ieskf_evaluation_patterns(oracle, epsi, max_iter):
    """Convergence limits and iteration caps that make the IESKF loop converge early, late or never
    give every redo / reuse evaluation pattern; the update matches the oracle (counts identical,
    pose within 1e-5) and the context is usable right after."""
    scene, m, scans = synth.make_config("C1", n_scans=2)
    om = oracle.OracleMap(m)
    tree = F.IkdTreeGPU()
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm, max_iteration=max_iter, epsi=epsi)
    for sc in scans:
        hm.set_scan(sc.body)
        st = synth.initial_state(sc.pos_init, sc.rot_init)
        P0 = synth.initial_cov()
        xg, Pg, sg = kf.update_iterated_dyn_share_modified(st, P0)
        xo, Po, so, _ = oracle.ieskf_update(om, sc.body, st, P0, max_iter=max_iter, limit=epsi)
        assert sg["h_evals"] == int(so[0]) and sg["knn_calls"] == int(so[1]) and sg["n_eff"] == int(so[3])
        assert sg["converged"] == int(so[2])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        np.testing.assert_allclose(Pg, Po, rtol=1e-5, atol=1e-10)
        assert hm(synth.pose24(xg), converge=True)[27] > 0
    hm.close()


def test_sums_handoff_under_load(c1):
    """The result hand-off (last block -> host-mapped sums + sequence number,
    write-through stores, no system release) checked word for word under
    uneven load: 300 rounds of redo/reuse evaluations at two alternating poses
    while another map + ctx on its own stream keeps the GPU busy from a second
    host thread.  Every returned sums vector must equal, bit for bit, the one
    the same evaluation gave on an idle GPU; a stale word (the previous
    evaluation's) would differ."""
    _, m, scans = c1
    sc = scans[0]
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    pa = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
    pb = pa.copy()
    pb[9:12] += np.array([0.05, -0.03, 0.02])  # translation

    def round_trip():
        return [hm(pa, True), hm(pa, False), hm(pb, True), hm(pb, False)]

    want = round_trip()
    assert not np.array_equal(want[0], want[2])  # the poses give different sums

    busy_tree = F.IkdTreeGPU(cell_size=1.0)
    busy_tree.Build(m)
    busy = F.HShareModelGPU(busy_tree)
    busy.set_scan(scans[1].body)
    stop = threading.Event()

    def load():
        k = 0
        while not stop.is_set():
            busy(pa, k % 3 == 0)
            k += 1

    th = threading.Thread(target=load)
    th.start()
    try:
        for it in range(300):
            got = round_trip()
            for g, w in zip(got, want):
                assert np.array_equal(g, w), f"round {it}: stale or torn sums"
    finally:
        stop.set()
        th.join()


@pytest.mark.parametrize("n_pts", [120_001, 200_000])
def test_h_model_many_blocks_matches_oracle(oracle, n_pts):
    """Scan sizes whose plane / reuse grids (469, 782 blocks) leave the last block's partial
    gather a multi-batch masked tail: sums of a redo and a reuse evaluation against the
    oracle (C2 map, the C2 scan repeated with a small offset to reach n_pts)."""
    _, m, scans = synth.make_config("C2", n_scans=1)
    sc = scans[0]
    reps = -(-n_pts // len(sc.body))
    body = np.concatenate([sc.body + np.float32(0.013 * k) for k in range(reps)])[:n_pts].astype(np.float32)
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    hm.set_scan(body)
    p24 = synth.pose24(synth.initial_state(sc.pos_init, sc.rot_init))
    om = oracle.OracleMap(m)
    o_redo, nn, sel, planes = _oracle_eval(oracle, om, body, p24)
    _check_sums(hm(p24, True), o_redo)
    p2 = p24.copy()
    p2[9:12] += np.array([0.02, -0.01, 0.005])
    o_reuse, _, _, _ = _oracle_eval(oracle, om, body, p2, nn, sel, planes, redo=False)
    _check_sums(hm(p2, False), o_reuse)


def test_icp_c4_multi_iteration_matches_oracle(oracle):
    """C4 at full size with a 2.5 m / 4 deg initial offset: 9 PCL iterations (each pass starting from the
    previous correspondences); transform within 1e-5, iterations and convergence state identical."""
    src, dst, _ = synth.make_icp_pair(n_points=500_000, seed=4321, disp=(2.5, 4.0))
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    lc.icpAlignment(src, dst)
    r = lc.last_result
    o = oracle.icp_align(src, dst)
    assert r.iterations == o["iterations"] >= 5 and r.state == o["state"]
    np.testing.assert_allclose(_T(r), o["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, o["fitness"], rtol=1e-5)
