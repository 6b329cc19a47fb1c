"""GPU parity of the incremental map against the oracle.

Bars: the map content (every id's xyz + alive flag) bit-exact after each
Add_Points / Delete_Point_Boxes / map_incremental; the reference's counters
equal; kNN over the updated map bit-exact (ids + sq-distances).
"""
import numpy as np
import pytest

from lio_gpu import frontend as F
from lio_gpu import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene_scans():
    scene, m, scans = synth.make_config("C1", n_scans=4)
    return scene, m, scans


def _same_map(tree, om):
    gx, ga = tree.by_id()
    ox, oa = om.by_id()
    assert gx.shape == ox.shape
    np.testing.assert_array_equal(ga, oa)
    np.testing.assert_array_equal(gx, ox)
    assert tree.size() == om.size()


def _knn_parity(tree, om, q):
    hm = F.HShareModelGPU(tree)
    hm.set_scan(q)  # identity pose: world = body
    p24 = np.zeros(24)
    p24[0:9] = np.eye(3).ravel()
    p24[12:21] = np.eye(3).ravel()
    hm(p24, True)
    gi, gd = hm.nearest_points()
    oi, od = om.knn(q, 5, 5.0)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd, od)
    hm.close()


def test_add_points_downsample_parity(oracle, scene_scans):
    _, m, scans = scene_scans
    base = m[:60000]
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    for k, sc in enumerate(scans[:3]):
        w = oracle.body_to_world(synth.pose24(synth.initial_state(sc.pos_gt, sc.rot_gt)), sc.body)
        c_gpu = tree.Add_Points(w, True)
        c_orc = om.add(w, True, 0.5)
        assert c_gpu == c_orc
        _same_map(tree, om)
    assert om.num_ids() > om.size()  # replaced points became tombstones
    _knn_parity(tree, om, scans[3].body + np.float32([3.0, 1.0, 0.0]))


def test_add_points_scrambled_order(oracle, scene_scans):
    """Voxels whose points are spread over many of the grouped update's 1024-point sort blocks (input
    order shuffled): the runs are re-ordered per voxel, so counters and map stay bit-exact."""
    _, m, scans = scene_scans
    base = m[:50000]
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    rng = np.random.default_rng(11)
    w = np.concatenate([oracle.body_to_world(synth.pose24(synth.initial_state(sc.pos_gt, sc.rot_gt)), sc.body)
                        for sc in scans[:3]])
    w = w[rng.permutation(len(w))]
    # <= 32 sort blocks: every voxel stays on the run-list path (up to 32 runs re-ordered per voxel)
    part = np.concatenate([w[:28000], w[:4000]])  # exact duplicates later in the order (ties on the centre distance)
    assert tree.Add_Points(part, True) == om.add(part, True, 0.5)
    _same_map(tree, om)
    rest = w[28000:]  # all of it: dense voxels may span > 64 blocks (the sorted fallback)
    assert tree.Add_Points(rest, True) == om.add(rest, True, 0.5)
    _same_map(tree, om)


def test_add_points_voxel_over_many_blocks(oracle, scene_scans):
    """One voxel offered 150k points (> 64 sort blocks of 1024): the grouped update is abandoned on the device
    and redone through the globally sorted path — same result."""
    _, m, _ = scene_scans
    base = m[:20000]
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    rng = np.random.default_rng(5)
    c = np.floor(base[123] / 0.5) * 0.5
    pts = (c + rng.uniform(0.01, 0.49, size=(150_000, 3))).astype(np.float32)
    pts[1000:1100] = pts[10]  # repeated points
    assert tree.Add_Points(pts, True) == om.add(pts, True, 0.5)
    _same_map(tree, om)
    small = (c + np.float32([2.0, 0.0, 0.0]) + rng.uniform(0.0, 0.5, size=(3000, 3))).astype(np.float32)
    assert tree.Add_Points(small, True) == om.add(small, True, 0.5)  # the grouped path again afterwards
    _same_map(tree, om)


def test_add_points_plain_and_delete_boxes(oracle, scene_scans):
    _, m, scans = scene_scans
    base = m[:40000]
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    extra = m[40000:52000]
    assert tree.Add_Points(extra, False) == len(extra)
    om.add(extra, False)
    _same_map(tree, om)
    lo, hi = base.min(0), base.max(0)
    mid = (lo + hi) / 2
    boxes = np.array([[lo[0] - 1, lo[1] - 1, lo[2] - 1, mid[0], mid[1], hi[2] + 1],
                      [mid[0] + 5, lo[1] - 1, lo[2] - 1, mid[0] + 20, hi[1] + 1, mid[2]]], np.float32)
    n_gpu = tree.Delete_Point_Boxes(boxes)
    n_orc = om.delete_boxes(boxes)
    assert n_gpu == n_orc > 0
    _same_map(tree, om)
    q = base[::97] + np.float32([0.05, -0.03, 0.02])
    _knn_parity(tree, om, q)


def test_add_outside_grid_rebuilds(oracle, scene_scans):
    _, m, _ = scene_scans
    base = m[:20000]
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    far = base[:3000] + np.float32([500.0, -300.0, 40.0])  # leaves the grid: full rebuild path
    assert tree.Add_Points(far, True) == om.add(far, True, 0.5)
    _same_map(tree, om)
    _knn_parity(tree, om, far[::7] + np.float32([0.1, 0.1, 0.0]))


def test_map_incremental_parity(oracle, scene_scans):
    """Scan-to-map sequence: build from the first scan, then per scan an IESKF
    update on the GPU followed by map_incremental; the oracle replays
    map_incremental with the same kNN pose / final pose."""
    _, _, scans = scene_scans
    sc0 = scans[0]
    p0 = synth.pose24(synth.initial_state(sc0.pos_gt, sc0.rot_gt))
    first = oracle.body_to_world(p0, sc0.body)
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(first)
    om = oracle.OracleDynMap(first)
    for sc in scans[1:]:
        hm = F.HShareModelGPU(tree)
        hm.set_scan(sc.body)
        kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
        x, P, st = kf.update_iterated_dyn_share_modified(synth.initial_state(sc.pos_init, sc.rot_init),
                                                         synth.initial_cov())
        p_knn = hm.last_knn_pose24()
        p_fin = synth.pose24(x)
        s_gpu = hm.map_incremental(p_fin, 0.5)
        s_orc = om.map_incremental(sc.body, p_knn, p_fin, 0.5, 0.5)
        assert s_gpu == s_orc
        _same_map(tree, om)
        hm.close()
    assert s_orc["n_to_add"] > 0


def test_everything_deleted_then_regrown(oracle, scene_scans):
    """Delete_Point_Boxes over the whole map: Nearest_Search finds nothing (no
    effective points, sums zero, empty lists); map_incremental then re-adds the
    scan through the downsampled Add_Points, as the oracle does."""
    _, m, scans = scene_scans
    base = m[:30000]
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    lo, hi = base.min(0) - 1, base.max(0) + 1
    box = np.array([[lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]]], np.float32)
    assert tree.Delete_Point_Boxes(box) == om.delete_boxes(box) == len(base)
    assert tree.size() == 0
    sc = scans[1]
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    p24 = synth.pose24(synth.initial_state(sc.pos_gt, sc.rot_gt))
    sums = hm(p24, True)
    assert not np.any(sums)
    gi, _ = hm.nearest_points()
    assert np.all(gi == -1)
    s_gpu = hm.map_incremental(p24, 0.5)
    s_orc = om.map_incremental(sc.body, p24, p24, 0.5, 0.5)
    assert s_gpu == s_orc and s_gpu["n_to_add"] == len(sc.body)
    _same_map(tree, om)
    hm.close()
    _knn_parity(tree, om, scans[2].body)


def test_nearest_search_batch(oracle, scene_scans):
    """ikd-Tree Nearest_Search over a batch (lio_map_nearest_search): k = 1..5,
    bounded and unbounded, after deletions (tombstoned ids) — ids and
    sq-distances bit-exact against the oracle, including far-away queries."""
    _, m, scans = scene_scans
    base = m[:50000]
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    lo, hi = base.min(0), base.max(0)
    mid = (lo + hi) / 2
    box = np.array([[lo[0] - 1, lo[1] - 1, lo[2] - 1, mid[0], mid[1], hi[2] + 1]], np.float32)
    assert tree.Delete_Point_Boxes(box) == om.delete_boxes(box) > 0
    rng = np.random.default_rng(3)
    q = np.concatenate([scans[1].body[::5],
                        rng.uniform(lo - 20, hi + 20, (3000, 3)).astype(np.float32)]).astype(np.float32)
    for k in (1, 3, 5):
        for max_dist in (float("inf"), 2.0, 0.3):
            gi, gd = tree.Nearest_Search(q, k, max_dist)
            oi, od = om.knn(q, k, max_dist * max_dist)
            np.testing.assert_array_equal(gi, oi)
            np.testing.assert_array_equal(gd, od)
    gi, _ = tree.Nearest_Search(q, 5)
    assert np.all(gi[:, 4] >= 0)  # unbounded: always 5 over a 25k-point map


def test_long_drive_with_fov_segment(oracle):
    """A 30-scan drive along the street, per scan as laserMapping runs it: lasermap_fov_segment
    (a small local cube so its deletes fire), the IESKF update on the GPU, map_incremental. The
    oracle replays the deletes and map_incremental with the same kNN / final poses: the map
    content stays bit-exact through every scan (tombstones, grid rebuilds, id growth)."""
    _, _, scans = synth.make_config("C1", n_scans=30, scan_points=8192)
    sc0 = scans[0]
    first = oracle.body_to_world(synth.pose24(synth.initial_state(sc0.pos_gt, sc0.rot_gt)), sc0.body)
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(first)
    om = oracle.OracleDynMap(first)
    lm = F.LocalMap(cube_len=200.0, det_range=30.0)
    deleted = 0
    errs = []
    for sc in scans[1:]:
        st = synth.initial_state(sc.pos_init, sc.rot_init)
        pos_lid = st["pos"] + synth.quat_to_mat(st["rot"]) @ synth.T_LI
        boxes = lm.update(pos_lid)
        if len(boxes):
            n = tree.Delete_Point_Boxes(boxes)
            assert n == om.delete_boxes(boxes)
            deleted += n
        hm = F.HShareModelGPU(tree)
        hm.set_scan(sc.body)
        kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
        x, _, _ = kf.update_iterated_dyn_share_modified(st, synth.initial_cov())
        p_knn, p_fin = hm.last_knn_pose24(), synth.pose24(x)
        assert hm.map_incremental(p_fin, 0.5) == om.map_incremental(sc.body, p_knn, p_fin, 0.5, 0.5)
        _same_map(tree, om)
        hm.close()
        errs.append(np.linalg.norm(x["pos"] - sc.pos_gt))
    assert deleted > 0  # the local-map cube moved at least once
    # no ground-truth map here (it is grown from the estimates, as in FAST-LIO): only check that the
    # odometry stays sane; the parity above is the point of the test
    assert np.all(np.isfinite(errs)) and max(errs) < 1.0
    _knn_parity(tree, om, scans[-1].body + np.float32([1.0, 0.5, 0.0]))


@pytest.mark.parametrize("headroom,dirty", [(64, 0), (0, 3), (64, 3)])
def test_pool_and_tombstone_list_recovery(oracle, scene_scans, headroom, dirty):
    """the gapped grid's two recovery paths — the slot pool exhausted while a cell moves to a
    bigger block (flag 2) and the per-update list of cells holding tombstones full (flag 4) — each end in a
    full re-lay from by_id.  Forced here with a pool capped at (slots in use + headroom) and a 3-cell list:
    Add_Points with downsample (replacements -> tombstones) and map_incremental stay bit-exact against the
    oracle, the rebuild counter goes up with the flags, and the kNN over the re-laid grid is exact."""
    _, m, scans = scene_scans
    base = m[:60000]
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(base)
    om = oracle.OracleDynMap(base)
    tree.set_test_limits(headroom, dirty)
    r0 = tree.stats()["rebuilds"]
    seen = 0
    for sc in scans[:3]:
        w = oracle.body_to_world(synth.pose24(synth.initial_state(sc.pos_gt, sc.rot_gt)), sc.body)
        assert tree.Add_Points(w, True) == om.add(w, True, 0.5)
        seen |= tree.stats()["flags"]
        _same_map(tree, om)
    sc = scans[3]
    hm = F.HShareModelGPU(tree)
    hm.set_scan(sc.body)
    kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
    x, _, _ = kf.update_iterated_dyn_share_modified(synth.initial_state(sc.pos_init, sc.rot_init), synth.initial_cov())
    p_knn, p_fin = hm.last_knn_pose24(), synth.pose24(x)
    assert hm.map_incremental(p_fin, 0.5) == om.map_incremental(sc.body, p_knn, p_fin, 0.5, 0.5)
    seen |= tree.stats()["flags"]
    hm.close()
    _same_map(tree, om)
    want = (2 if headroom else 0) | (4 if dirty else 0)
    assert seen & want == want, (seen, want)
    assert tree.stats()["rebuilds"] > r0
    _knn_parity(tree, om, scans[0].body + np.float32([2.0, -1.0, 0.0]))
