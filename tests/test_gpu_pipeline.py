"""The C5 stream end to end, loop leg included (BASELINE.json configs[4]).

Eight raw 120 k-point KITTI-64 sweeps on the 10 M-point C5 map — four driving out, four driving back
30 s later — go through the GPU front end (lio_gpu.pipeline.FastLioSamStream: Preprocess +
UndistortPcl + downSizeFilterSurf -> IESKF update -> map_incremental -> keyframe) and, independently,
through the oracle chained from ITS OWN outputs (its preprocess, its IESKF, its map_incremental with
its own poses, its keyframes).  Then fast_lio_sam's loop leg on the newest keyframe
(fast_lio_sam.cpp:682-730): fetchClosestKeyframeIdx -> setSrcAndDstCloud -> icpAlignment
(loop_closure.cpp:18-126).

Bars:
* per sweep: feats_down_body and feats_undistort bit-exact; pose within 1e-5; evaluation counts equal;
  the keyframe cloud made on the GPU bit-exact against the numpy glue (pointBodyToWorld + transformPcd);
* the loop candidate index equal;
* stage parity on the GPU's keyframes: submaps bit-exact, ICP transform within 1e-5, iterations and
  convergence state identical, fitness score within 1e-5 relative;
* chained parity: the oracle's ICP on its own submaps against the GPU's — transform within 1e-5,
  iterations identical.
"""
import numpy as np
import pytest

from lio_gpu import frontend as F
from lio_gpu import loop_closure as LC
from lio_gpu import pipeline as PL
from lio_gpu import synth

pytestmark = pytest.mark.gpu


def _T(r):
    return np.array(list(r.T), np.float32).reshape(4, 4)


@pytest.mark.timeout(900)
def test_c5_stream_with_loop_closure(oracle):
    mp, L, sp, kind = synth.CONFIGS["C5"]
    scene = synth.make_scene(L, 1234)
    m = synth.sample_surface(scene, mp, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0, downsample_size=0.5)
    tree.Build(m)
    cfg = LC.LoopClosureConfig()
    gs = PL.FastLioSamStream(tree, cfg)
    om = oracle.OracleDynMap(m)
    P0 = synth.initial_cov()
    kfo = []
    for k, (raw, poses, end24, st0, t) in enumerate(synth.make_loop_stream(scene)):
        g = gs.process(raw, poses, end24, st0, P0, t)
        o_down = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.5)
        o_und = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.0)
        assert g["n_down"] == len(o_down) > 1000
        np.testing.assert_array_equal(gs.hm.undistorted(), o_und)
        body = np.ascontiguousarray(o_down[:, :3])
        xo, Po, so, _, xk = oracle.ieskf_update(om.tree(), body, st0, P0, knn_state=True)
        xg, sg = g["state"], g["stats"]
        # the keyframe cloud built on the GPU (lio_scan_keyframe_cloud) = the numpy glue, bit for bit
        kh = gs.keyframe_host(xg, t, k)
        np.testing.assert_array_equal(gs.keyframes[-1].pcd_, kh.pcd_)
        np.testing.assert_array_equal(gs.keyframes[-1].pose_eig_, kh.pose_eig_)
        if k == 0:  # a matrix-only pose (no quaternions): q / q_LI derived from R / R_LI, same cloud
            Tk = PL.odom_matrix(xg)
            p_mat = F.pose_from_pose24(np.asarray(synth.pose24(xg), np.float64)[:24])
            assert not any(p_mat.q) and not any(p_mat.q_LI)
            # (the derived quaternion may differ from the state's in its last bits: float-store tolerance)
            np.testing.assert_allclose(gs.hm.keyframe_cloud(p_mat, np.linalg.inv(Tk)), gs.keyframes[-1].pcd_,
                                       rtol=0, atol=1e-4)
        assert sg["h_evals"] == int(so[0]) and sg["knn_calls"] == int(so[1]) and sg["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        assert np.linalg.norm(xg["pos"] - end24[9:12]) < 0.2
        om.map_incremental(body, synth.pose24(xk), synth.pose24(xo), 0.5, 0.5)  # the oracle's own poses
        w_o = oracle.body_to_world(synth.pose24(xo), o_und[:, :3])
        # the host glue's pointBodyToWorld is the restatement's, bit for bit
        np.testing.assert_array_equal(PL.state_world(xo, o_und[:, :3]), w_o)
        kfo.append(PL.keyframe_from_odometry(xo, np.concatenate([w_o, o_und[:, 3:4]], axis=1), t, k))
    # the loop leg on the newest keyframe (submap_range 2: the out and back legs' own neighbourhoods)
    idx, out_g, _ = gs.loop(submap_range=2)
    assert idx == gs.lc.fetchClosestKeyframeIdx(kfo[-1], kfo) == 0
    r = gs.lc.last_result
    src_g, dst_g = gs.lc.src_cloud_, gs.lc.dst_cloud_
    assert len(src_g) > 5_000 and len(dst_g) > 5_000

    def submaps(kfs, center):
        ids = [i for i in range(center - 2, center + 3) if 0 <= i < len(kfs) - 1]
        return oracle.submap_voxelize([kfs[i].pcd_ for i in ids], [kfs[i].pose_corrected_eig_ for i in ids], cfg.voxel_res_)

    # stage parity: the GPU's keyframes through the oracle
    np.testing.assert_array_equal(src_g, submaps(gs.keyframes, len(gs.keyframes) - 1))
    np.testing.assert_array_equal(dst_g, submaps(gs.keyframes, idx))
    o = oracle.icp_align(src_g[:, :3], dst_g[:, :3])
    assert r.iterations == o["iterations"] >= 1 and r.state == o["state"]
    np.testing.assert_allclose(_T(r), o["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, o["fitness"], rtol=1e-5)
    assert out_g.is_valid_ == o["is_valid"] and out_g.is_valid_
    # chained parity: the oracle's own stream
    src_o, dst_o = submaps(kfo, len(kfo) - 1), submaps(kfo, idx)
    assert abs(len(src_o) - len(src_g)) <= 0.001 * len(src_g) and abs(len(dst_o) - len(dst_g)) <= 0.001 * len(dst_g)
    oc = oracle.icp_align(src_o[:, :3], dst_o[:, :3])
    assert oc["iterations"] == r.iterations and oc["state"] == r.state
    np.testing.assert_allclose(_T(r), oc["T"], atol=1e-5)
    np.testing.assert_allclose(r.score, oc["fitness"], rtol=1e-4)
    gs.close()
