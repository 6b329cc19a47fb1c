"""Point-cloud filters, CPU side: the C restatement
(oracle/lio_oracle.cpp voxel_grid / transform_segments / preprocess) against
naive numpy/Python restatements of PCL 1.10 VoxelGrid::applyFilter,
pcl::transformPointCloud<double> and FAST-LIO Preprocess + UndistortPcl [U].
Parity with the real reference is unpinned (PCL is not installed; FAST-LIO is
an empty submodule), so these pin the restatement against a second reading.
"""
import math

import numpy as np

import oracle_py as O

f32 = np.float32


def py_voxel_grid(pts, leaf):
    pts = np.asarray(pts, f32)
    leaf = np.broadcast_to(np.asarray(leaf, f32), 3)
    fin = np.all(np.isfinite(pts[:, :3]), axis=1)
    q = pts[fin]
    if len(q) == 0:
        return np.zeros((0, pts.shape[1]), f32)
    inv = (f32(1.0) / leaf).astype(f32)
    lo, hi = q[:, :3].min(0), q[:, :3].max(0)
    min_b = np.floor(lo * inv).astype(np.int64)
    max_b = np.floor(hi * inv).astype(np.int64)
    div = max_b - min_b + 1
    if div[0] * div[1] * div[2] > 2**31 - 1:
        return pts.copy()
    mul = np.array([1, div[0], div[0] * div[1]])
    ijk = (np.floor(q[:, :3] * inv).astype(f32) - min_b.astype(f32)).astype(np.int64)
    idx = ijk @ mul
    order = np.argsort(idx, kind="stable")
    out = []
    j = 0
    while j < len(order):
        e = j
        acc = np.zeros(pts.shape[1], f32)
        while e < len(order) and idx[order[e]] == idx[order[j]]:
            acc = (acc + q[order[e]]).astype(f32)
            e += 1
        out.append((acc / f32(e - j)).astype(f32))
        j = e
    return np.array(out, f32)


def test_voxel_grid_matches_python():
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.uniform(-5, 5, (3000, 3)), rng.uniform(0, 100, (3000, 1))], axis=1).astype(f32)
    pts[::97, 1] = np.nan  # non-finite rows are dropped
    for leaf in (0.3, 0.5, [0.4, 0.7, 1.1]):
        a = O.voxel_grid(pts, leaf)
        b = py_voxel_grid(pts, leaf)
        np.testing.assert_array_equal(a, b)
    # clusters: many points per voxel exercise the in-order sums
    c = (rng.normal(0, 0.05, (2000, 4)) + np.repeat(rng.uniform(-2, 2, (20, 4)), 100, axis=0)).astype(f32)
    np.testing.assert_array_equal(O.voxel_grid(c, 0.5), py_voxel_grid(c, 0.5))


def test_voxel_grid_overflow_returns_input():
    pts = np.array([[0, 0, 0], [1e6, 1e6, 1e6], [5, 5, 5]], f32)
    np.testing.assert_array_equal(O.voxel_grid(pts, 1e-3), pts)


def test_submap_voxelize_matches_python():
    rng = np.random.default_rng(4)
    clouds = [np.concatenate([rng.uniform(-3, 3, (500, 3)), rng.uniform(0, 50, (500, 1))], axis=1).astype(f32)
              for _ in range(4)]
    poses = []
    for k in range(4):
        a = 0.3 * k
        T = np.eye(4)
        T[:3, :3] = [[math.cos(a), -math.sin(a), 0], [math.sin(a), math.cos(a), 0], [0, 0, 1]]
        T[:3, 3] = [1.5 * k, -0.7 * k, 0.1 * k]
        poses.append(T)
    tf = []
    for c, T in zip(clouds, poses):
        x = c[:, :3].astype(np.float64)
        y = np.empty_like(c)
        for r in range(3):  # ((m0 x + m1 y) + m2 z) + m3 in double, stored float
            y[:, r] = (((T[r, 0] * x[:, 0] + T[r, 1] * x[:, 1]) + T[r, 2] * x[:, 2]) + T[r, 3]).astype(f32)
        y[:, 3] = c[:, 3]
        tf.append(y)
    ref = py_voxel_grid(np.concatenate(tf), 0.3)
    np.testing.assert_array_equal(O.submap_voxelize(clouds, poses, 0.3), ref)


def _exp(w, dt):
    nrm = math.sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2])
    E = np.eye(3)
    if not nrm > 1e-7:
        return E
    r = np.asarray(w) / nrm
    K = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
    a = nrm * dt
    return E + math.sin(a) * K + ((1.0 - math.cos(a)) * K) @ K


def py_preprocess(raw, poses, end, every=4, blind=2.0, leaf=0.5):
    """Preprocess + UndistortPcl (literal backward loop incl. its first-point quirk) + VoxelGrid."""
    sel = [raw[i] for i in range(len(raw)) if i % every == 0 and
           f32(f32(f32(raw[i, 0] * raw[i, 0]) + f32(raw[i, 1] * raw[i, 1])) + f32(raw[i, 2] * raw[i, 2])) > f32(blind * blind)]
    pts = np.array(sel, f32)
    pts = pts[np.argsort(pts[:, 4], kind="stable")]
    R_end, p_end = end[0:9].reshape(3, 3), end[9:12]
    R_LI, t_LI = end[12:21].reshape(3, 3), end[21:24]
    it = len(pts) - 1
    for kp in range(len(poses) - 1, 0, -1):
        hd, tl = poses[kp - 1], poses[kp]
        while float(pts[it, 4]) / 1000.0 > hd["offset_time"]:
            dt = float(pts[it, 4]) / 1000.0 - hd["offset_time"]
            Ri = np.asarray(hd["rot"]) @ _exp(tl["gyr"], dt)
            Tei = hd["pos"] + hd["vel"] * dt + 0.5 * tl["acc"] * dt * dt - p_end
            P = pts[it, :3].astype(np.float64)
            c = R_LI.T @ (R_end.T @ (Ri @ (R_LI @ P + t_LI) + Tei) - t_LI)
            pts[it, :3] = c.astype(f32)
            if it == 0:
                break
            it -= 1
    return py_voxel_grid(pts, leaf) if leaf > 0 else pts


def _scene_scan(n=8000, seed=11):
    from lio_gpu import synth

    scene = synth.make_scene(200.0, 1234)
    return synth.make_raw_scan(scene, n, seed=seed)


def test_preprocess_matches_python():
    raw, poses, end = _scene_scan()
    for leaf in (0.0, 0.5):
        a = O.preprocess(raw, poses, end, leaf=leaf)
        b = py_preprocess(raw, poses, end, leaf=leaf)
        assert a.shape == b.shape
        # numpy's matrix products may pair the double sums differently: compare to 1 float ulp
        np.testing.assert_allclose(a, b, rtol=2e-7, atol=1e-6)
    # the first-point quirk: earliest point past the first IMU sample -> compensated by every older segment
    raw2 = raw[raw[:, 4] > 35.0]
    a = O.preprocess(raw2, poses, end, point_filter_num=1, leaf=0.0)
    b = py_preprocess(raw2, poses, end, every=1, leaf=0.0)
    np.testing.assert_allclose(a, b, rtol=2e-7, atol=1e-6)


def test_pipeline_glue_world_transform_matches_restatement(oracle):
    """lio_gpu.pipeline.state_world (the keyframe glue's pointBodyToWorld, numpy in Eigen's operation
    order) equals the restatement's body_to_world bit for bit; transform_pcd round-trips through
    odom_matrix's inverse to within float rounding."""
    from lio_gpu import pipeline as PL
    from lio_gpu import synth

    rng = np.random.default_rng(0)
    for _ in range(4):
        st = synth.initial_state(rng.normal(size=3) * 50, synth.rotvec_to_quat(rng.normal(size=3)))
        xyz = (rng.normal(size=(20000, 3)) * 30).astype(np.float32)
        w = PL.state_world(st, xyz)
        np.testing.assert_array_equal(w, oracle.body_to_world(synth.pose24(st), xyz))
        T = PL.odom_matrix(st)
        back = PL.transform_pcd(np.concatenate([w, xyz[:, :1]], axis=1), np.linalg.inv(T))
        ref = (xyz.astype(np.float64) @ synth.quat_to_mat(st["offset_R_L_I"]).T + st["offset_T_L_I"])
        np.testing.assert_allclose(back[:, :3], ref, atol=1e-4)
        np.testing.assert_array_equal(back[:, 3], xyz[:, 0])


def test_eigen_inverse4_is_an_inverse():
    """lio_gpu.pipeline.eigen_inverse4 (Eigen 3.3's SSE Matrix4d::inverse restated) inverts general and
    rigid 4x4 matrices to the last bits (structure check of the restatement: a misplaced lane or sign would
    not give an inverse)."""
    from lio_gpu import pipeline as PL

    rng = np.random.default_rng(11)
    for _ in range(20):
        M = rng.normal(size=(4, 4))
        np.testing.assert_allclose(PL.eigen_inverse4(M) @ M, np.eye(4), rtol=0, atol=1e-12)
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        T = PL.odom_matrix(dict(rot=q, pos=rng.uniform(-50, 50, 3)))
        np.testing.assert_allclose(PL.eigen_inverse4(T), np.linalg.inv(T), rtol=0, atol=1e-13)
