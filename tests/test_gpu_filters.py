"""GPU parity of the point-cloud filters against the oracle.

Bars: VoxelGrid and transformPcd + voxelizePcd bit-exact (same float op order,
input order inside a voxel); scan preprocessing (Preprocess + UndistortPcl +
downSizeFilterSurf) bit-exact — the undistortion's sin / cos are one fixed-order
routine on both sides (lio_filter.hip / lio_oracle.cpp sincos_fixed).
"""
import math

import numpy as np
import pytest

from lio_gpu import filters as FL
from lio_gpu import frontend as F
from lio_gpu import loop_closure as LC
from lio_gpu import synth

pytestmark = pytest.mark.gpu
f32 = np.float32


def test_voxel_grid_bit_exact(oracle):
    rng = np.random.default_rng(21)
    vg = FL.VoxelGrid(0.5)
    for stride in (3, 4, 5, 8):
        pts = rng.uniform(-30, 30, (200_000, stride)).astype(f32)
        pts[:, 2] *= 0.1
        pts[::1013, 0] = np.nan
        for leaf in (0.3, 0.5, 2.0):
            vg.setLeafSize(leaf, leaf, leaf)
            np.testing.assert_array_equal(vg.filter(pts), oracle.voxel_grid(pts, leaf))
    # clustered (many points per voxel), anisotropic leaf
    c = (rng.normal(0, 0.05, (50_000, 4)) + np.repeat(rng.uniform(-5, 5, (500, 4)), 100, axis=0)).astype(f32)
    vg.setLeafSize(0.2, 0.4, 0.3)
    np.testing.assert_array_equal(vg.filter(c), oracle.voxel_grid(c, [0.2, 0.4, 0.3]))
    # index overflow: PCL returns the input
    big = np.array([[0, 0, 0], [1e6, 1e6, 1e6], [5, 5, 5]], f32)
    vg.setLeafSize(1e-3, 1e-3, 1e-3)
    np.testing.assert_array_equal(vg.filter(big), big)


@pytest.mark.parametrize("n", [1, 2, 1023, 4096, 4097, 32767, 32768, 32769, 40000])
def test_voxel_grid_sizes_around_one_block_runs(oracle, n):
    """The run bounds of <= 32768 sorted keys come from one block (voxel_runs_block_kernel: 8 tiles of 4096,
    loads up front, ballot prefix), larger inputs from run_head + the device scan + voxel_bounds; both feed
    the one-wave-per-voxel centroids.  Bit-exact on either side of the switch, with long runs (> 64 points
    per voxel: chunked sums) and NaN rows mixed in."""
    rng = np.random.default_rng(n)
    pts = rng.uniform(-20, 20, (n, 4)).astype(f32)
    k = max(n // 200, 1)
    pts[: 100 * k] = (rng.normal(0, 0.02, (min(100 * k, n), 4)) + np.repeat(rng.uniform(-5, 5, (k, 4)), 100, axis=0)[: min(100 * k, n)]).astype(f32)
    pts[1::997, 1] = np.nan
    vg = FL.VoxelGrid(0.5)
    np.testing.assert_array_equal(vg.filter(pts), oracle.voxel_grid(pts, 0.5))


def test_submap_voxelize_bit_exact(oracle):
    scene, m, scans = synth.make_config("C1", n_scans=6)
    rng = np.random.default_rng(5)
    kfs = []
    for k, sc in enumerate(scans):
        pcd = np.concatenate([sc.body, rng.uniform(0, 255, (len(sc.body), 1))], axis=1).astype(f32)
        T = np.eye(4)
        T[:3, :3] = synth.quat_to_mat(sc.rot_gt)
        T[:3, 3] = sc.pos_gt
        kfs.append(LC.PosePcd(pcd_=pcd, pose_corrected_eig_=T))
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    src, dst = lc.setSrcAndDstCloud(kfs, src_idx=4, dst_idx=1, submap_range=2, voxel_res=0.3)
    # reference loop: i in [idx - range, idx + range], 0 <= i < keyframes.size() - 1 (newest excluded)
    def ref(center):
        ids = [i for i in range(center - 2, center + 3) if 0 <= i < len(kfs) - 1]
        return oracle.submap_voxelize([kfs[i].pcd_ for i in ids], [kfs[i].pose_corrected_eig_ for i in ids], 0.3)
    np.testing.assert_array_equal(src, ref(4))
    np.testing.assert_array_equal(dst, ref(1))
    # the voxelized submaps feed icpAlignment (xyz of PointXYZI rows)
    out = lc.icpAlignment(src, dst)
    assert np.isfinite(out.score_)


def _close(a, b):
    assert a.shape == b.shape
    np.testing.assert_array_equal(a, b)


def test_preprocess_matches_oracle(oracle):
    scene = synth.make_scene(400.0, 1234)
    raw, poses, end24 = synth.make_raw_scan(scene, 120_000, seed=3)
    end = F.pose_from_pose24(end24)
    for leaf in (0.0, 0.5):
        pp = FL.ScanPreprocessor(point_filter_num=4, blind=2.0, filter_size_surf=leaf, time_field=4)
        g = pp.process(raw, poses, end)
        o = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=leaf)
        _close(g, o)
    # earliest point past the first IMU sample: the reference's repeated compensation of the first point
    raw2 = raw[raw[:, 4] > 35.0]
    pp = FL.ScanPreprocessor(point_filter_num=1, blind=2.0, filter_size_surf=0.0, time_field=4)
    _close(pp.process(raw2, poses, end), oracle.preprocess(raw2, poses, end24, point_filter_num=1, leaf=0.0))


def test_scan_preprocess_into_ctx(oracle):
    """Raw scan -> feats_down_body on the device -> h_share_model, without a host round trip."""
    scene = synth.make_scene(400.0, 1234)
    raw, poses, end24 = synth.make_raw_scan(scene, 120_000, seed=4)
    m = synth.sample_surface(scene, 200_000, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    n = hm.preprocess_scan(raw, poses, F.pose_from_pose24(end24), point_filter_num=4, blind=2.0,
                           filter_size_surf=0.5, time_field=4)
    o = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.5)
    assert n == len(o) > 0
    p24 = np.zeros(24)
    p24[0:9] = np.eye(3).ravel()
    p24[12:21] = np.eye(3).ravel()
    hm(p24, True)
    np.testing.assert_array_equal(hm.world(), o[:, :3])


def test_preprocess_staged_upload_edges(oracle):
    """The staged upload (Preprocess's selection made while the host packs the rows, one DMA), the single
    host wait, the time sort skipped for rows already in time order and the learnt voxel-key width: ragged
    row counts, wider records, shuffled times (sorted path), non-finite rows and negative times, nothing
    selected, one row, a small extent followed by a large one (the learnt key width too narrow: the call
    repeats at full width), VoxelGrid's index overflow (output = the undistorted input) and the staging
    buffer growing and shrinking between calls — each bit-exact against the oracle, through the filter API
    and into a ctx (feats_down_body and feats_undistort)."""
    scene = synth.make_scene(400.0, 1234)
    raw, poses, end24 = synth.make_raw_scan(scene, 120_000, seed=8)
    end = F.pose_from_pose24(end24)
    rng = np.random.default_rng(3)
    wide = np.concatenate([raw[:, :4], rng.uniform(0, 1, (len(raw), 1)).astype(f32), raw[:, 4:5]], axis=1)
    m = synth.sample_surface(scene, 100_000, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    hm = F.HShareModelGPU(tree)
    near = raw[np.linalg.norm(raw[:, :3], axis=1) < 6.0][:800]      # a small extent: few voxel-key bits learnt
    shuffled = raw[rng.permutation(len(raw))[:50_000]]               # times out of order: the sorted path
    holes = raw[:30_000].copy()
    holes[::97, 1] = np.nan                                          # non-finite rows (never selected)
    holes[5::211, 4] = -holes[5::211, 4]                             # negative times
    cases = [(near, 1, 2.0, 0.5, 4), (raw[:120_001 - 7], 3, 2.0, 0.5, 4), (near, 2, 2.0, 0.5, 4),
             (shuffled, 2, 2.0, 0.5, 4), (holes, 1, 2.0, 0.5, 4), (raw[:5_000], 4, 2.0, 0.5, 4),
             (wide[:60_017], 5, 2.0, 0.5, 5), (raw[:1], 1, 0.0, 0.5, 4), (raw[:2_000], 4, 1e4, 0.5, 4),
             (raw[:40_000], 2, 2.0, 1e-4, 4), (raw, 4, 2.0, 0.0, 4), (raw[:777], 7, 2.0, 0.3, 4)]
    for rows, every, blind, leaf, tf in cases:
        end_tf = end
        o_down = oracle.preprocess(rows, poses, end24, point_filter_num=every, blind=blind, leaf=leaf, time_field=tf)
        o_und = oracle.preprocess(rows, poses, end24, point_filter_num=every, blind=blind, leaf=0.0, time_field=tf)
        pp = FL.ScanPreprocessor(point_filter_num=every, blind=blind, filter_size_surf=leaf, time_field=tf)
        _close(pp.process(rows, poses, end_tf), o_down)
        n = hm.preprocess_scan(rows, poses, end_tf, point_filter_num=every, blind=blind, filter_size_surf=leaf,
                               time_field=tf)
        assert n == len(o_down), (len(rows), every, blind, leaf)
        _close(hm.undistorted(), o_und)
        if n:
            p24 = np.zeros(24)
            p24[0:9] = np.eye(3).ravel()
            p24[12:21] = np.eye(3).ravel()
            hm(p24, True)
            np.testing.assert_array_equal(hm.world(), o_down[:, :3])
