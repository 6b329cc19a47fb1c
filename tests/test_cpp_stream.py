"""The C5 stream driven from C++: tests/cpp/c5_stream.cpp runs
lio_gpu::FastLioSamStream (include/lio_gpu.hpp) over the same eight raw KITTI-64 sweeps on the 10 M-point
C5 map as tests/test_gpu_pipeline.py — preprocess -> IESKF update -> map_incremental -> keyframe, then the
loop leg on the newest keyframe (fast_lio_sam.cpp:367-573,682-730; loop_closure.cpp:18-126) — and this test
checks its output against the oracle chained from its own outputs:

* per sweep: feats_down_body size and feats_undistort size equal the oracle's; pose within 1e-5; the IESKF
  evaluation counts equal; the keyframe cloud equal to the numpy glue (pointBodyToWorld + transformPcd with
  the C++ pose inverse: within 2 float ulps, the two 4x4 inverses differ in the last bits);
* the loop candidate index equal to the oracle's;
* stage parity: the C++ submaps bit-exact against the oracle's submap_voxelize of the C++ keyframes, the ICP
  transform within 1e-5, iterations and convergence state identical, fitness within 1e-5 relative;
* chained parity: the oracle's ICP on its own submaps within 1e-5 of the C++ transform.
"""
import os
import subprocess

import numpy as np
import pytest

from lio_gpu import pipeline as PL
from lio_gpu import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "fast-lio-sam_gps_amd", "lio_gpu", "_lib")
SRC = os.path.join(ROOT, "tests", "cpp", "c5_stream.cpp")


def test_c5_stream_driver_compiles(tmp_path):
    assert os.path.exists(os.path.join(LIBDIR, "liblio_gpu.so")), "build the library first (make -C fast-lio-sam_gps_amd)"
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), SRC, "-o", str(tmp_path / "c5_stream"),
           "-L", LIBDIR, "-llio_gpu", "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]


def test_host_glue_matches_python(tmp_path):
    """odom_matrix (bit for bit), inverse4 (bit for bit against the Python restatement of Eigen's SSE
    Matrix4d::inverse, and within 1e-14 of numpy's inverse) and fetch_closest_keyframe_idx of the C++ header
    against the Python glue — host code only, no GPU."""
    import re

    from lio_gpu import loop_closure as LC

    exe = str(tmp_path / "glue")
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "test_host_glue.cpp"), "-o", exe,
           "-L", LIBDIR, "-llio_gpu", "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60).stdout
    T = np.array([float(v) for v in re.findall(r"^T \d+ (\S+)$", out, re.M)]).reshape(4, 4)
    Ic = np.array([float(v) for v in re.findall(r"^I \d+ (\S+)$", out, re.M)]).reshape(4, 4)
    st = dict(rot=np.array([0.9238795325112867, 0.0123, -0.0456, 0.3826834323650898]), pos=np.array([12.5, -3.25, 0.75]))
    np.testing.assert_array_equal(T, PL.odom_matrix(st))
    np.testing.assert_array_equal(Ic, PL.eigen_inverse4(T))
    np.testing.assert_allclose(Ic, np.linalg.inv(T), rtol=0, atol=1e-14)
    np.testing.assert_allclose(Ic @ T, np.eye(4), rtol=0, atol=1e-14)
    kfs = []
    for k in range(8):
        P = np.eye(4)
        P[0, 3] = 3.7 * k if k < 4 else 3.7 * (7 - k) + 1.5
        P[1, 3] = 0.0 if k < 4 else -0.3
        kfs.append(LC.PosePcd(pcd_=np.zeros((0, 4), np.float32), pose_corrected_eig_=P,
                              timestamp_=0.1 * k if k < 4 else 40.0 + 0.1 * (k - 4), idx_=k))
    lco = LC.LoopClosure.__new__(LC.LoopClosure)  # host logic only: no handle
    lco.config_ = LC.LoopClosureConfig()
    want = lco.fetchClosestKeyframeIdx(kfs[-1], kfs)
    assert int(re.search(r"^closest (-?\d+)$", out, re.M).group(1)) == want == 0
    assert int(re.search(r"^closest_early (-?\d+)$", out, re.M).group(1)) == lco.fetchClosestKeyframeIdx(kfs[3], kfs[:4]) == -1


def test_stream_io_round_trip(tmp_path):
    """The input writer's layout (read back field by field) — host glue only."""
    import struct

    scene = synth.make_scene(200.0, 5)
    m = synth.sample_surface(scene, 1000, 5)
    stream = synth.make_loop_stream(scene, n_out=1, n_points=2000)
    p = str(tmp_path / "in.bin")
    PL.write_stream_input(p, m, stream, synth.initial_cov(), 3)
    b = open(p, "rb").read()
    assert b[:8] == b"LIOC5IN1" and struct.unpack_from("<q", b, 8)[0] == len(m)
    o = 16 + 12 * len(m)
    assert struct.unpack_from("<i", b, o)[0] == len(stream)
    raw = stream[0][0]
    assert struct.unpack_from("<qi", b, o + 4) == raw.shape
    assert struct.unpack_from("<i", b, len(b) - 4)[0] == 3


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_cpp_c5_stream_matches_oracle(oracle, tmp_path):
    mp, L, sp, kind = synth.CONFIGS["C5"]
    scene = synth.make_scene(L, 1234)
    m = synth.sample_surface(scene, mp, 1234)
    stream = synth.make_loop_stream(scene)
    P0 = synth.initial_cov()
    fin, fout = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    PL.write_stream_input(fin, m, stream, P0, submap_range=2)
    summary = PL.run_cpp_stream(fin, fout)
    print(summary)
    out = PL.read_stream_output(fout)
    assert len(out["sweeps"]) == len(stream)
    om = oracle.OracleDynMap(m)
    kfo = []
    for k, ((raw, poses, end24, st0, t), g) in enumerate(zip(stream, out["sweeps"])):
        o_down = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.5)
        o_und = oracle.preprocess(raw, poses, end24, point_filter_num=4, blind=2.0, leaf=0.0)
        assert g["n_down"] == len(o_down) > 1000 and g["n_undistorted"] == len(o_und)
        body = np.ascontiguousarray(o_down[:, :3])
        xo, Po, so, _, xk = oracle.ieskf_update(om.tree(), body, st0, P0, knn_state=True)
        xg = g["state"]
        assert g["h_evals"] == int(so[0]) and g["knn_calls"] == int(so[1]) and g["n_eff"] == int(so[3])
        np.testing.assert_allclose(xg["pos"], xo["pos"], atol=1e-5)
        np.testing.assert_allclose(xg["rot"], xo["rot"], atol=1e-5)
        # the keyframe: /cloud_registered of the C++ state taken back by the C++ pose_eig_.inverse()
        T = PL.odom_matrix(xg)
        np.testing.assert_array_equal(g["pose_eig"], T)
        w_g = PL.state_world(xg, o_und[:, :3])
        kh = PL.keyframe_from_odometry(xg, np.concatenate([w_g, o_und[:, 3:4]], axis=1), t, k)
        np.testing.assert_array_equal(g["pcd"], kh.pcd_)  # the same Eigen inverse restated on both sides
        om.map_incremental(body, synth.pose24(xk), synth.pose24(xo), 0.5, 0.5)  # the oracle's own poses
        w_o = oracle.body_to_world(synth.pose24(xo), o_und[:, :3])
        kfo.append(PL.keyframe_from_odometry(xo, np.concatenate([w_o, o_und[:, 3:4]], axis=1), t, k))
    lp = out["loop"]
    from lio_gpu import loop_closure as LC

    cfg = LC.LoopClosureConfig()
    lco = LC.LoopClosure.__new__(LC.LoopClosure)  # fetchClosestKeyframeIdx is host logic: no handle needed
    lco.config_ = cfg
    assert lp["closest_idx"] == lco.fetchClosestKeyframeIdx(kfo[-1], kfo) == 0

    def submaps(clouds, poses, center):
        ids = [i for i in range(center - 2, center + 3) if 0 <= i < len(clouds) - 1]
        return oracle.submap_voxelize([clouds[i] for i in ids], [poses[i] for i in ids], cfg.voxel_res_)

    gc = [s["pcd"] for s in out["sweeps"]]
    gp = [s["pose_eig"] for s in out["sweeps"]]
    src_g, dst_g = lp["src"], lp["dst"]
    assert len(src_g) > 5_000 and len(dst_g) > 5_000
    np.testing.assert_array_equal(src_g, submaps(gc, gp, len(gc) - 1))
    np.testing.assert_array_equal(dst_g, submaps(gc, gp, lp["closest_idx"]))
    o = oracle.icp_align(src_g[:, :3], dst_g[:, :3])
    assert lp["iterations"] == o["iterations"] >= 1 and lp["state"] == o["state"]
    np.testing.assert_allclose(lp["T"], o["T"], atol=1e-5)
    np.testing.assert_allclose(lp["score"], o["fitness"], rtol=1e-5)
    assert lp["is_valid"] == o["is_valid"] and lp["is_valid"]
    src_o = submaps([kf.pcd_ for kf in kfo], [kf.pose_corrected_eig_ for kf in kfo], len(kfo) - 1)
    dst_o = submaps([kf.pcd_ for kf in kfo], [kf.pose_corrected_eig_ for kf in kfo], lp["closest_idx"])
    oc = oracle.icp_align(src_o[:, :3], dst_o[:, :3])
    assert oc["iterations"] == lp["iterations"]
    np.testing.assert_allclose(lp["T"], oc["T"], atol=1e-5)
    # the C++ preprocess stage (<= 0.15 ms per sweep) is reported, not asserted here
    assert summary["sweeps"] == len(stream) and summary["stage_ms_median"]["preprocess"] > 0


def test_loop_sequence_driver_compiles(tmp_path):
    """tests/cpp/loop_sequence.cpp (the loop leg as the node runs it) builds against the C++ mirror with -Werror."""
    assert os.path.exists(os.path.join(LIBDIR, "liblio_gpu.so")), "build the library first (make -C fast-lio-sam_gps_amd)"
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "loop_sequence.cpp"),
           "-o", str(tmp_path / "loop_sequence"), "-L", LIBDIR, "-llio_gpu", "-Wl,-rpath," + LIBDIR,
           "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_cpp_loop_sequence_matches_python_and_oracle(oracle, tmp_path):
    """The loop leg as fast_lio_sam's loopTimerFunc runs it (fast_lio_sam.cpp:682-728), from C++: one
    LoopClosure handle, the keyframe database growing by one keyframe per call, a drifted return leg.  Every
    call's closest keyframe, submap sizes, iterations and transform equal the Python LoopClosure's on the same
    keyframes bit for bit; two calls' ICP is within 1e-5 of the oracle (PCL float order 2) on the C++ submaps
    recomputed by the Python glue; after the first call the handle allocates nothing (lio_alloc_count)."""
    from lio_gpu import loop_closure as LC

    kfs = PL.make_loop_keyframes(n_out=8, n_back=8, n0=12_000, dn=600)
    calls = list(range(8, 16))
    fin = str(tmp_path / "ls.bin")
    PL.write_loop_sequence(fin, kfs, calls)
    out = PL.run_loop_sequence(fin, timeout=600)
    print({k: v for k, v in out.items() if k != "per_call"})
    assert out["calls"] == len(calls) and out["warm_allocs"] == 0
    lc = LC.LoopClosure(LC.LoopClosureConfig())
    for c, k in zip(out["per_call"], calls):
        keyframes = kfs[:k + 1]
        closest = lc.fetchClosestKeyframeIdx(keyframes[-1], keyframes)
        assert c["k"] == k and c["closest"] == closest >= 0
        reg = lc.performLoopClosure(keyframes[-1], keyframes, closest)
        assert (c["n_src"], c["n_dst"]) == (len(lc.src_cloud_), len(lc.dst_cloud_))
        assert c["iterations"] == lc.last_result.iterations >= 1 and c["valid"] == reg.is_valid_
        np.testing.assert_array_equal(c["T"], np.array(list(lc.last_result.T), np.float32).reshape(4, 4))
        if k in (calls[0], calls[-1]):
            o = oracle.icp_align(np.ascontiguousarray(lc.src_cloud_[:, :3]), np.ascontiguousarray(lc.dst_cloud_[:, :3]),
                                 params=oracle.default_icp_params())
            assert o["iterations"] == c["iterations"]
            np.testing.assert_allclose(c["T"], o["T"], atol=1e-5)
    lc.close()
