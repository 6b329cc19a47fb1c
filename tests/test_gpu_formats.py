"""GPU parity of the wire / disk formats: byte work, bit-exact
against numpy's own structured-array decoding / encoding."""
import numpy as np
import pytest

from lio_gpu import filters as FL
from lio_gpu import formats as FM
from lio_gpu import frontend as F
from lio_gpu import synth

pytestmark = pytest.mark.gpu


def _ouster_like(n, rng, big_endian=False):
    """x y z (f32), intensity (f32), t (u32 ns), reflectivity (u16), ring (u8), range (u32), a f64 column."""
    e = ">" if big_endian else "<"
    dt = np.dtype({"names": ["x", "y", "z", "intensity", "t", "refl", "ring", "range", "d"],
                   "formats": [e + "f4", e + "f4", e + "f4", e + "f4", e + "u4", e + "u2", "u1", e + "u4", e + "f8"],
                   "offsets": [0, 4, 8, 16, 20, 24, 26, 28, 32], "itemsize": 48})
    a = np.zeros(n, dt)
    a["x"], a["y"], a["z"] = rng.normal(0, 20, (3, n))
    a["intensity"] = rng.uniform(0, 300, n)
    a["t"] = rng.integers(0, 100_000_000, n)
    a["refl"] = rng.integers(0, 65535, n)
    a["ring"] = rng.integers(0, 128, n)
    a["range"] = rng.integers(0, 2**32 - 1, n, dtype=np.uint64)
    a["d"] = rng.normal(0, 1e3, n)
    return a


def test_cloud2_decode_bit_exact():
    rng = np.random.default_rng(2)
    cc = FM.CloudCodec()
    for be in (False, True):
        a = _ouster_like(50_000, rng, be)
        fields = [(0, FM.FLOAT32), (4, FM.FLOAT32), (8, FM.FLOAT32), (16, FM.FLOAT32), (20, FM.UINT32, 1e-6),
                  (24, FM.UINT16), (26, FM.UINT8), (32, FM.FLOAT64)]
        out = cc.decode(a.tobytes(), len(a), 48, fields, big_endian=be)
        exp = np.stack([a["x"].astype(np.float32), a["y"].astype(np.float32), a["z"].astype(np.float32),
                        a["intensity"].astype(np.float32),
                        (a["t"].astype(np.float32) * np.float32(1e-6)).astype(np.float32),
                        a["refl"].astype(np.float32), a["ring"].astype(np.float32),
                        a["d"].astype(np.float32)], axis=1)
        np.testing.assert_array_equal(out, exp)
    # absent field -> 0
    out = cc.decode(a.tobytes(), len(a), 48, [(0, FM.FLOAT32), (0, 0)], big_endian=True)
    assert np.all(out[:, 1] == 0)


def test_cloud2_encode_pointxyzi():
    rng = np.random.default_rng(3)
    rec = rng.normal(0, 5, (10_000, 4)).astype(np.float32)
    cc = FM.CloudCodec()
    data = cc.encode(rec)
    dt = np.dtype({"names": ["x", "y", "z", "intensity"], "formats": ["<f4"] * 4, "offsets": [0, 4, 8, 16],
                   "itemsize": 32})
    exp = np.zeros(len(rec), dt)
    for k, nm in enumerate(dt.names):
        exp[nm] = rec[:, k]
    assert data == exp.tobytes()
    np.testing.assert_array_equal(cc.decode(data, len(rec), 32, [(o, t) for o, t in FM.POINTXYZI[0]]), rec)


def test_pcd_roundtrip_and_map_build(tmp_path, oracle):
    rng = np.random.default_rng(4)
    rec = rng.uniform(-50, 50, (30_000, 4)).astype(np.float32)
    p = str(tmp_path / "map.pcd")
    FM.write_pcd_binary(p, rec)
    cc = FM.CloudCodec()
    np.testing.assert_array_equal(cc.read_pcd(p), rec)
    np.testing.assert_array_equal(cc.read_pcd(p, ("z", "x", "nope")), np.stack([rec[:, 2], rec[:, 0], 0 * rec[:, 0]], 1))
    pa = str(tmp_path / "a.pcd")
    with open(pa, "w") as f:
        f.write("# .PCD v0.7\nVERSION 0.7\nFIELDS x y z intensity\nSIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\n"
                f"WIDTH {len(rec)}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {len(rec)}\nDATA ascii\n")
        for r in rec[:500]:
            f.write(" ".join(repr(float(v)) for v in r) + "\n")
    with open(pa) as f:  # fix the count to the rows written
        txt = f.read().replace(f"POINTS {len(rec)}", "POINTS 500").replace(f"WIDTH {len(rec)}", "WIDTH 500")
    open(pa, "w").write(txt)
    np.testing.assert_array_equal(cc.read_pcd(pa), rec[:500])
    # saved map -> GPU grid -> kNN parity
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build_pcd(p)
    np.testing.assert_array_equal(tree.points(), rec[:, :3])


def test_scan_preprocess_from_cloud2_matches_records():
    scene = synth.make_scene(400.0, 1234)
    raw, poses, end24 = synth.make_raw_scan(scene, 60_000, seed=9)
    # Velodyne-like PointCloud2: x y z intensity (f32) + time (f32 seconds) at offset 20, point_step 32
    dt = np.dtype({"names": ["x", "y", "z", "intensity", "time"], "formats": ["<f4"] * 5,
                   "offsets": [0, 4, 8, 16, 20], "itemsize": 32})
    a = np.zeros(len(raw), dt)
    for k, nm in enumerate(["x", "y", "z", "intensity"]):
        a[nm] = raw[:, k]
    a["time"] = raw[:, 4] / np.float32(1000.0)
    fields = [(0, FM.FLOAT32), (4, FM.FLOAT32), (8, FM.FLOAT32), (16, FM.FLOAT32), (20, FM.FLOAT32, 1000.0)]
    m = synth.sample_surface(scene, 100_000, 1234)
    tree = F.IkdTreeGPU(cell_size=1.0)
    tree.Build(m)
    end = F.pose_from_pose24(end24)
    h1 = F.HShareModelGPU(tree)
    n1 = h1.preprocess_cloud2(a.tobytes(), len(a), 32, fields, poses, end)
    # the same records through the float path (time column recovered exactly as the decoder does)
    rec = np.concatenate([raw[:, :4], (a["time"] * np.float32(1000.0))[:, None]], axis=1).astype(np.float32)
    h2 = F.HShareModelGPU(tree)
    n2 = h2.preprocess_scan(rec, poses, end)
    assert n1 == n2 > 0
    p24 = np.zeros(24)
    p24[0:9] = np.eye(3).ravel()
    p24[12:21] = np.eye(3).ravel()
    h1(p24, True)
    h2(p24, True)
    np.testing.assert_array_equal(h1.world(), h2.world())
