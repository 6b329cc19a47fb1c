"""CPU tests of the oracle (oracle/lio_oracle.cpp) against independent implementations.

The reference ships no tests or golden vectors for this path (SURVEY.md §4,
§8c), so the restatement is cross-checked here against scipy's cKDTree, numpy
brute force, numpy least squares and numpy's SVD-based Umeyama.
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from lio_gpu import synth


def _bf_knn(m, q, k, r2):
    """Brute force in the oracle's float op order, total order (d2, id)."""
    out_i = np.full((len(q), k), -1, np.int32)
    out_d = np.full((len(q), k), np.inf, np.float32)
    for j, p in enumerate(q):
        dx = (p[0] - m[:, 0]).astype(np.float32)
        dy = (p[1] - m[:, 1]).astype(np.float32)
        dz = (p[2] - m[:, 2]).astype(np.float32)
        d = (dx * dx + dy * dy) + dz * dz
        ok = np.nonzero(d <= np.float32(r2))[0]
        o = ok[np.lexsort((ok, d[ok]))][:k]
        out_i[j, :len(o)] = o
        out_d[j, :len(o)] = d[o]
    return out_i, out_d


def test_knn_vs_bruteforce_with_ties(oracle):
    rng = np.random.default_rng(0)
    m = rng.uniform(-3, 3, (3000, 3)).astype(np.float32)
    m = np.concatenate([m, m[:200]])  # exact duplicates -> distance ties broken by lower id
    q = rng.uniform(-3.5, 3.5, (400, 3)).astype(np.float32)
    q[:50] = m[:50]  # queries on map points (d2 = 0, duplicated)
    om = oracle.OracleMap(m)
    for k, r2 in ((5, 5.0), (5, 0.05), (1, np.inf), (8, 1.0)):
        idx, d2 = om.knn(q, k=k, range_sq=r2)
        bi, bd = _bf_knn(m, q, k, r2)
        np.testing.assert_array_equal(idx, bi)
        np.testing.assert_array_equal(d2, bd)


def test_knn_vs_ckdtree_c1(oracle):
    scene, m, scans = synth.make_config("C1", n_scans=1)
    om = oracle.OracleMap(m)
    st = synth.initial_state(scans[0].pos_init, scans[0].rot_init)
    w = oracle.body_to_world(synth.pose24(st), scans[0].body)
    idx, d2 = om.knn(w, 5, 5.0)
    tr = cKDTree(m.astype(np.float64))
    dd, ii = tr.query(w.astype(np.float64), k=5, distance_upper_bound=np.sqrt(5.0) * (1 + 1e-6))
    full = (idx[:, 4] >= 0) & np.isfinite(dd[:, 4])
    assert full.mean() > 0.95
    # identical neighbour sets (scipy works in float64, ordering can differ only on near-ties)
    same = np.all(np.sort(idx[full], 1) == np.sort(ii[full], 1), axis=1)
    assert same.mean() > 0.9999
    # distances are the float32 formula
    mm = m[idx[full]]
    ww = w[full][:, None, :]
    ref = ((ww[..., 0] - mm[..., 0]) ** 2 + (ww[..., 1] - mm[..., 1]) ** 2) + (ww[..., 2] - mm[..., 2]) ** 2
    np.testing.assert_array_equal(d2[full], ref.astype(np.float32))
    assert np.all(np.diff(d2[full], axis=1) >= 0)


def test_esti_plane_vs_lstsq(oracle):
    rng = np.random.default_rng(1)
    for trial in range(300):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        d = rng.uniform(-20, 20)
        # 5 points near the plane n.x + d = 0
        base = rng.uniform(-30, 30, 3)
        base -= (n @ base + d) * n
        u = np.cross(n, [1, 0, 0] if abs(n[0]) < 0.9 else [0, 1, 0])
        u /= np.linalg.norm(u)
        v = np.cross(n, u)
        P = base + rng.uniform(-0.5, 0.5, (5, 1)) * u + rng.uniform(-0.5, 0.5, (5, 1)) * v
        P += rng.normal(0, 0.005, (5, 1)) * n
        P = P.astype(np.float32)
        ok, out = oracle.esti_plane(P, 0.1)
        x, *_ = np.linalg.lstsq(P.astype(np.float64), -np.ones(5), rcond=None)
        nn = np.linalg.norm(x)
        ref = np.concatenate([x / nn, [1 / nn]])
        if np.abs(P.astype(np.float64) @ ref[:3] + ref[3]).max() > 0.09:
            continue  # ill-conditioned A n = -1 (plane near the origin): even the f64 fit fails the gate
        assert ok
        np.testing.assert_allclose(out, ref, rtol=2e-3, atol=2e-4)
        # unit normal
        assert abs(np.linalg.norm(out[:3].astype(np.float64)) - 1) < 1e-5


def test_esti_plane_rejects_non_planar(oracle):
    rng = np.random.default_rng(2)
    P = rng.uniform(-1, 1, (5, 3)).astype(np.float32) + np.float32(5)
    ok, _ = oracle.esti_plane(P, 0.1)
    assert not ok


def test_h_share_model_sums_consistent(oracle):
    scene, m, scans = synth.make_config("C1", n_scans=1)
    om = oracle.OracleMap(m)
    sc = scans[0]
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    p24 = synth.pose24(st)
    n = len(sc.body)
    nn = np.full((n, 5), -1, np.int32)
    sel = np.zeros(n, np.uint8)
    planes = np.zeros((n, 4), np.float32)
    sums = oracle.h_share_model(om, sc.body, p24, True, nn, sel, planes)
    k = sel.astype(bool)
    assert int(sums[27]) == k.sum() > 0.5 * n
    # rebuild H in numpy from the per-point outputs (float64) and compare
    R = p24[:9].reshape(3, 3)
    pI = sc.body[k].astype(np.float64) + synth.T_LI
    nrm = planes[k, :3].astype(np.float64)
    C = nrm @ R  # R^T n per row
    A = np.cross(pI, C)
    J = np.concatenate([nrm, A], 1)
    h = -planes[k, 3].astype(np.float64)
    HTH = J.T @ J
    iu = np.triu_indices(6)
    np.testing.assert_allclose(sums[:21], HTH[iu], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(sums[21:27], J.T @ h, rtol=1e-8, atol=1e-9)
    np.testing.assert_allclose(sums[28], np.abs(planes[k, 3]).astype(np.float64).sum(), rtol=1e-12)


def test_ieskf_converges_to_ground_truth(oracle):
    scene, m, scans = synth.make_config("C1", n_scans=1)
    om = oracle.OracleMap(m)
    sc = scans[0]
    st = synth.initial_state(sc.pos_init, sc.rot_init)
    x, P, stats, _ = oracle.ieskf_update(om, sc.body, st, synth.initial_cov())
    err0 = np.linalg.norm(sc.pos_init - sc.pos_gt)
    err1 = np.linalg.norm(x["pos"] - sc.pos_gt)
    assert err1 < 0.2 * err0
    q = x["rot"]
    assert abs(np.linalg.norm(q) - 1) < 1e-9
    ang = 2 * np.arccos(min(1.0, abs(q @ sc.rot_gt)))
    assert ang < np.deg2rad(0.1)
    assert stats[0] <= 4 and stats[1] >= 1
    # covariance shrinks and stays symmetric PSD
    assert np.all(np.diag(P)[:6] < np.diag(synth.initial_cov())[:6])
    np.testing.assert_allclose(P, P.T, atol=1e-12)
    assert np.linalg.eigvalsh(0.5 * (P + P.T)).min() > -1e-12


def _umeyama_np(src, dst):
    mu_s, mu_d = src.mean(0), dst.mean(0)
    S = (dst - mu_d).T @ (src - mu_s) / len(src)
    U, s, Vt = np.linalg.svd(S)
    D = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        D[2, 2] = -1
    R = U @ D @ Vt
    return R, mu_d - R @ mu_s


def test_icp_first_step_matches_numpy_umeyama(oracle):
    src, dst, T = synth.make_icp_pair(n_points=20000, seed=11)
    res = oracle.icp_align(src, dst, params=oracle.double_icp_params())  # the double form vs numpy's SVD
    # first iteration: correspondences = unbounded 1-NN within 52.5 m
    tr = cKDTree(dst.astype(np.float64))
    d, i = tr.query(src.astype(np.float64))
    keep = d <= 52.5
    R, t = _umeyama_np(src[keep].astype(np.float64), dst[i[keep]].astype(np.float64))
    T1 = res["trace"][0, 2:18].reshape(4, 4)
    np.testing.assert_allclose(T1[:3, :3], R, atol=2e-6)
    np.testing.assert_allclose(T1[:3, 3], t, atol=2e-5)
    assert res["converged"] and res["iterations"] >= 1
    # the recovered transform brings the clouds together (independent 0.3 m
    # voxelizations keep a residual floor, and PCL's configured criteria stop
    # once a step is < 0.1 m / 8 deg, loop_closure.cpp:8)
    assert res["fitness"] < res["trace"][0, 1]
    assert np.linalg.norm(res["T"][:3, 3] - T[:3, 3]) < np.linalg.norm(T[:3, 3])


def test_icp_not_enough_correspondences(oracle):
    src = np.array([[0, 0, 0], [1, 0, 0]], np.float32)
    dst = np.array([[100, 0, 0], [101, 0, 0], [100, 1, 0]], np.float32)
    res = oracle.icp_align(src, dst)
    assert not res["converged"] and res["state"] == 5 and res["iterations"] == 0


# ---------------------------------------------------------------------------
# SO3 * v as Eigen evaluates it (VERDICT r01 weak #2a): numpy transcription of
# Eigen 3.3 QuaternionBase::_transformVector, element-wise in float64 with the
# same operation order, compared bit for bit with the oracle's world points.
def _np_cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _np_transform_vector(q, v):
    """Eigen: uv = q.vec().cross(v); uv += uv; return v + q.w() * uv + q.vec().cross(uv)."""
    w, qv = q[0], (q[1], q[2], q[3])
    uv = _np_cross(qv, v)
    uv = tuple(u + u for u in uv)
    c = _np_cross(qv, uv)
    return tuple((v[i] + w * uv[i]) + c[i] for i in range(3))


def _np_mat_to_quat(m):
    """Eigen 3.3 quaternionbase_assign_impl<Other,3,3>: trace = m00 + (m11 + m22)."""
    t = m[0, 0] + (m[1, 1] + m[2, 2])
    c = [0.0] * 4  # x y z w
    if t > 0:
        t = np.sqrt(t + 1.0)
        c[3] = 0.5 * t
        t = 0.5 / t
        c[0] = (m[2, 1] - m[1, 2]) * t
        c[1] = (m[0, 2] - m[2, 0]) * t
        c[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        c[i] = 0.5 * t
        t = 0.5 / t
        c[3] = (m[k, j] - m[j, k]) * t
        c[j] = (m[j, i] + m[i, j]) * t
        c[k] = (m[k, i] + m[i, k]) * t
    return np.array([c[3], c[0], c[1], c[2]])


@pytest.mark.parametrize("from_matrix", [False, True])
def test_world_points_follow_eigen_transform_vector(oracle, from_matrix):
    """p_world = rot * (offset_R_L_I * p + t_LI) + pos (FAST-LIO pointBodyToWorld / h_share_model [U]),
    both products through _transformVector, stored as float.  Non-unit quaternions included (the
    state's quaternion is not renormalised between boxplus steps); with from_matrix the pose carries
    only matrices and the quaternions come from Eigen's Matrix3 -> Quaternion conversion."""
    rng = np.random.default_rng(42)
    body = rng.uniform(-60, 60, (4000, 3)).astype(np.float32)
    for trial in range(12):
        q = synth.rotvec_to_quat(rng.normal(0, 1.2, 3)) * (1.0 + (trial % 3) * 1e-7)
        qli = synth.rotvec_to_quat(rng.normal(0, 0.05, 3))
        if trial == 0:
            q = np.array([0.0, 0.0, 0.0, 1.0])  # trace < 0 branches of the matrix conversion
        t = rng.uniform(-500, 500, 3)
        tli = rng.normal(0, 0.5, 3)
        R, RLI = synth.quat_to_mat(q), synth.quat_to_mat(qli)
        if from_matrix:
            p = np.concatenate([R.ravel(), t, RLI.ravel(), tli])  # no quaternions: derived from R
            q, qli = _np_mat_to_quat(R), _np_mat_to_quat(RLI)
        else:
            p = np.concatenate([R.ravel(), t, RLI.ravel(), tli, q, qli])
        w = oracle.body_to_world(p, body)
        b = tuple(body[:, i].astype(np.float64) for i in range(3))
        a = _np_transform_vector(qli, b)
        a = tuple(a[i] + tli[i] for i in range(3))
        g = _np_transform_vector(q, a)
        ref = np.stack([g[i] + t[i] for i in range(3)], axis=1).astype(np.float32)
        np.testing.assert_array_equal(w, ref)


def test_icp_float_umeyama_mode_close_to_double(oracle):
    """Fidelity study (VERDICT r01 weak #2b): the oracle's float restatement of pcl::umeyama (float
    sums, Eigen JacobiSVD) against the double-statistics form the GPU path computes.  They agree to
    PCL's own float noise (DESIGN.md §2 lists the measured gaps: ~2e-5 at 8k-30k points, ~2e-4 at
    500k), and take the same iterations / convergence state."""
    for n, seed in ((8000, 3), (30000, 5)):
        src, dst, _ = synth.make_icp_pair(n_points=n, seed=seed)
        rd = oracle.icp_align(src, dst, params=oracle.double_icp_params())
        p = oracle.default_icp_params()
        p.umeyama_float = 1
        rf = oracle.icp_align(src, dst, params=p)
        assert rd["iterations"] == rf["iterations"] and rd["state"] == rf["state"]
        np.testing.assert_allclose(rf["T"], rd["T"], atol=1e-4)
        assert abs(rf["fitness"] - rd["fitness"]) <= 1e-4 * rd["fitness"]


def test_sincos_fixed_within_one_ulp(oracle):
    """UndistortPcl's sin / cos in the restatement: one fixed-order routine (fdlibm algorithm) that the
    GPU evaluates identically; pinned here against numpy (libm) to <= 1 ulp (1e-30 absolute next to
    the zeros), equal in > 80 % of the samples."""
    rng = np.random.default_rng(11)
    a = np.concatenate([rng.uniform(-1e-3, 1e-3, 20000), rng.uniform(-1, 1, 50000), rng.uniform(-50, 50, 50000),
                        [0.0, -0.0, 1e-30, np.pi / 4, 0.3, 0.78125, np.pi / 2, np.pi, 3 * np.pi / 2, 1e5]])
    s, c = oracle.sincos(a)
    for got, ref in ((s, np.sin(a)), (c, np.cos(a))):
        # relative to 1 ulp, or (near the zeros of sin / cos, where the 3-part pi/2 reduction
        # cancels) to 1e-30 absolute
        ulp = np.maximum(np.spacing(np.abs(ref)), 1e-30)
        err = np.abs(got - ref) / ulp
        assert err.max() <= 1.0, err.max()
        assert np.mean(got == ref) > 0.8  # glibc rounds correctly more often; never by more than 1 ulp


def test_eigen_gemm_kc(oracle):
    """Eigen 3.3's depth blocking of a 3 x k by k x 3 float GEMM (SSE2 gebp: mr 8, nr 4, KcFactor 1):
    max_kc = ((l1 - mr nr 4) / (4 (mr + nr))) & ~7 = 680 (32 KiB L1) / 1016 (48 KiB), the last block made as
    large as possible; no blocking below 48 or up to max_kc."""
    assert oracle.eigen_gemm_kc(500_000, 32 * 1024) == 680
    assert oracle.eigen_gemm_kc(500_000, 48 * 1024) == 1016
    assert oracle.eigen_gemm_kc(3000, 32 * 1024) == 608  # 680 - 8 ((679 - 3000 % 680) // (8 (3000 // 680 + 1)))
    assert oracle.eigen_gemm_kc(680, 32 * 1024) == 680 and oracle.eigen_gemm_kc(47, 32 * 1024) == 47
    assert oracle.eigen_gemm_kc(1360, 32 * 1024) == 680


def _np_umeyama_sigma(src, tgt, order):
    """numpy float32 restatement of pcl::umeyama's means and sigma in summation order `order` (1: sequential,
    2 / 3: Eigen 3.3 GEMM blocking, 4 / 5: packet-4 means) — independent of lio_oracle.cpp."""
    import oracle_py as O

    f32 = np.float32
    n = len(src)
    oon = f32(1.0) / f32(n)

    def rsum(v):
        if order in (4, 5) and n >= 4:
            e2, e1 = (n // 8) * 8, (n // 4) * 4
            p0 = v[0:4].copy()
            if e1 > 4:
                p1 = v[4:8].copy()
                for i in range(8, e2, 8):
                    p0 = (p0 + v[i:i + 4]).astype(f32)
                    p1 = (p1 + v[i + 4:i + 8]).astype(f32)
                p0 = (p0 + p1).astype(f32)
                if e1 > e2:
                    p0 = (p0 + v[e2:e2 + 4]).astype(f32)
            a = f32(f32(p0[0] + p0[2]) + f32(p0[1] + p0[3]))
            for i in range(e1, n):
                a = f32(a + v[i])
            return a
        return np.cumsum(v, dtype=f32)[-1]

    sm = np.array([f32(rsum(src[:, d]) * oon) for d in range(3)], f32)
    dm = np.array([f32(rsum(tgt[:, d]) * oon) for d in range(3)], f32)
    prod = ((tgt - dm)[:, :, None] * (src - sm)[:, None, :]).astype(f32)  # [k, r, c], float products
    if order in (2, 3, 5):
        kc = O.eigen_gemm_kc(n, 48 * 1024 if order == 3 else 32 * 1024)
        sig = np.zeros((3, 3), f32)
        for k2 in range(0, n, kc):
            C0 = np.cumsum(prod[k2:k2 + kc], axis=0, dtype=f32)[-1]
            sig = (sig + (oon * C0).astype(f32)).astype(f32)
        return sm, dm, sig
    return sm, dm, (oon * np.cumsum(prod, axis=0, dtype=f32)[-1]).astype(f32)


def test_umeyama_float_orders_match_numpy(oracle):
    """Each float summation order of the oracle's pcl::umeyama (UmeyamaOrder 1-5) reproduces an independent
    numpy float32 restatement bit for bit: means (sequential / packet-4 redux) and sigma (one sequential
    depth sum scaled at the end / Eigen 3.3 GEMM blocks res += alpha * block sum).  Lengths below and above
    kc, the lazy-product threshold excepted (n >= 14)."""
    rng = np.random.default_rng(5)
    q = np.array([0.99, 0.05, -0.08, 0.1])
    R = synth.quat_to_mat(q / np.linalg.norm(q))
    for n in (14, 47, 700, 3000):
        src = (rng.standard_normal((n, 3)) * 20 + 5).astype(np.float32)
        tgt = (src @ R.T + np.array([1.0, -2.0, 0.5])).astype(np.float32) + rng.normal(0, 0.01, (n, 3)).astype(np.float32)
        sig = {}
        for order in range(1, 6):
            _, sm, dm, sg = oracle.umeyama_float(src, tgt, order, stats=True)
            nsm, ndm, nsg = _np_umeyama_sigma(src, tgt, order)
            np.testing.assert_array_equal(sm, nsm)
            np.testing.assert_array_equal(dm, ndm)
            np.testing.assert_array_equal(sg, nsg)
            sig[order] = sg
        if n > 680:
            assert not np.array_equal(sig[1], sig[2])  # the blocking changes sigma's bits


def test_umeyama_order_spread_pins_the_fidelity_bar(oracle):
    """how well is "PCL's float ICP result" defined?  The oracle's ICP (PCL 1.10 criteria) on a
    C4-shaped pair with every float summation order (lio_oracle.cpp UmeyamaOrder) and with the double
    statistics.  Measured at full size (500 k, scripts/umeyama_spread.py): the Eigen 3.3 orders
    (1-3: sequential means) agree to 3.2e-6 (pair A) / 3.8e-5 (pair B), the packet-mean orders differ by
    1.8e-4, and the double statistics sit 1.86e-4 / 1.2e-4 from the sequential-mean orders — outside the
    1e-5 bar, so the timed fidelity mode is order 2.  Here at 100 k (pair B): the same structure."""
    src, dst, _ = synth.make_icp_pair(n_points=100_000, seed=4321, disp=(2.5, 4.0))
    res = {}
    for order in range(0, 6):
        p = oracle.default_icp_params()
        p.umeyama_float = order
        res[order] = oracle.icp_align(src, dst, params=p)
    its = {o: (r["iterations"], r["state"]) for o, r in res.items()}
    assert len(set(its.values())) == 1, its

    def d(a, b):
        return float(np.abs(res[a]["T"] - res[b]["T"]).max())

    eigen33 = max(d(a, b) for a in (1, 2, 3) for b in (1, 2, 3))
    print(f"100k pair B: Eigen 3.3 orders spread {eigen33:.3g}; 2 vs 3 {d(2, 3):.3g}; double vs 2 {d(0, 2):.3g}; "
          f"packet vs sequential means {d(4, 1):.3g}")
    assert d(1, 2) > 0.0  # the GEMM blocking changes the result
    assert d(2, 3) < 1e-5  # the two L1 sizes agree to the bar
    assert eigen33 < 1e-4
    assert d(0, 2) < 1e-3


def test_undistort_libm_sincos_changes_no_point_at_c5(oracle):
    """the reference's UndistortPcl calls libm sin / cos; the restatement (and the
    GPU) evaluate one pinned fdlibm-order routine.  Over the C5 stream (8 raw KITTI-64 sweeps) the undistorted
    and the downsampled clouds are identical bit for bit under either: the Exp arguments |w| dt stay small
    (< 1e-3 rad), where the two agree exactly, and an ulp of a double product vanishes in the float store."""
    mp, L, sp, kind = synth.CONFIGS["C5"]
    scene = synth.make_scene(L, 1234)
    n_und = n_diff = 0
    try:
        for raw, poses, end24, st0, t in synth.make_loop_stream(scene):
            oracle.set_sincos_libm(False)
            a = oracle.preprocess(raw, poses, end24, leaf=0.0)
            ad = oracle.preprocess(raw, poses, end24, leaf=0.5)
            oracle.set_sincos_libm(True)
            b = oracle.preprocess(raw, poses, end24, leaf=0.0)
            bd = oracle.preprocess(raw, poses, end24, leaf=0.5)
            n_und += len(a)
            n_diff += int(np.count_nonzero(np.any(a.view(np.uint32) != b.view(np.uint32), axis=1)))
            assert len(ad) == len(bd)
            n_diff += int(np.count_nonzero(np.any(ad.view(np.uint32) != bd.view(np.uint32), axis=1)))
    finally:
        oracle.set_sincos_libm(False)
    assert n_und > 200_000
    assert n_diff == 0
