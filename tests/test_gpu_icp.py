"""Loop-closure ICP correspondence search on the GPU (icp_tile_kernel) vs brute force.

Every source point's 1-NN in the final (getFitnessScore) pass must be the exact
(d2, id)-minimum over the target, d2 = float ((dx*dx + dy*dy) + dz*dz) — the
kd-tree NN of PCL's KdTreeFLANN restated with the reference's total order
(oracle header, tests/oracle_py.py).  The aligned cloud the pass searched from
is `getFinalAlignedCloud()`, so the check needs no transform restatement.
Cases: the C4 shape at a small size, a source far outside the target (empty
surroundings: the geometric growth), a target of 1-3 points, exact ties, and
a multi-iteration alignment (later passes start from the previous
correspondence).
"""
import numpy as np
import pytest

from lio_gpu import loop_closure as LC
from lio_gpu import synth

pytestmark = pytest.mark.gpu


def brute_nn(q, t):
    """exact 1-NN under (d2, id), float32 d2 in the reference's operation order."""
    q = np.asarray(q, np.float32)
    t = np.asarray(t, np.float32)
    ids = np.empty(len(q), np.int32)
    d2 = np.empty(len(q), np.float32)
    for s in range(0, len(q), 2048):
        qq = q[s:s + 2048]
        dx = qq[:, None, 0] - t[None, :, 0]
        dy = qq[:, None, 1] - t[None, :, 1]
        dz = qq[:, None, 2] - t[None, :, 2]
        d = (dx * dx + dy * dy) + dz * dz  # float32 throughout, no FMA
        j = np.argmin(d, axis=1)  # first index of the minimum = lowest id among ties
        ids[s:s + 2048] = j
        d2[s:s + 2048] = d[np.arange(len(qq)), j]
    return ids, d2


def run(src, dst, cell=1.0, guess=None):
    lc = LC.LoopClosure(LC.LoopClosureConfig(), cell_size=cell)
    lc.setInputSource(src)
    lc.setInputTarget(dst)
    r = lc.align(guess=guess)
    ids, d2 = lc.correspondences()
    return lc, r, ids, d2


def check_nn(lc, ids, d2, dst):
    q = lc.getFinalAlignedCloud()
    bi, bd = brute_nn(q, dst)
    np.testing.assert_array_equal(d2, bd)
    np.testing.assert_array_equal(ids, bi)


@pytest.mark.parametrize("cell", [0.5, 1.0, 2.0])
def test_icp_nn_exact_c4_shape(cell):
    src, dst, _ = synth.make_icp_pair(n_points=20_000, seed=5)
    lc, r, ids, d2 = run(src, dst, cell)
    check_nn(lc, ids, d2, dst)


def test_icp_nn_source_far_outside_target():
    rng = np.random.default_rng(3)
    dst = rng.uniform(-5, 5, (4000, 3)).astype(np.float32)
    src = np.concatenate([rng.uniform(-5, 5, (3000, 3)),               # overlapping
                          rng.uniform(40, 60, (500, 3)),               # 40+ m away, one side
                          rng.uniform(-200, -150, (300, 3))]).astype(np.float32)
    lc, r, ids, d2 = run(src, dst, 1.0)
    check_nn(lc, ids, d2, dst)


@pytest.mark.parametrize("nt", [1, 3])
def test_icp_nn_tiny_target(nt):
    rng = np.random.default_rng(nt)
    dst = rng.uniform(-1, 1, (nt, 3)).astype(np.float32)
    src = rng.uniform(-30, 30, (5000, 3)).astype(np.float32)
    lc, r, ids, d2 = run(src, dst, 1.0)
    check_nn(lc, ids, d2, dst)


def test_icp_nn_ties_lowest_id():
    # target on an integer lattice, duplicated points: equal distances everywhere
    g = np.stack(np.meshgrid(np.arange(-4, 5), np.arange(-4, 5), np.arange(0, 3), indexing="ij"), -1).reshape(-1, 3)
    dst = np.concatenate([g, g[::-1]]).astype(np.float32)  # every point twice, different ids
    rng = np.random.default_rng(7)
    src = (rng.integers(-8, 9, (4000, 3)) * 0.5).astype(np.float32)  # half-integer: many exact ties
    lc, r, ids, d2 = run(src, dst, 1.0, guess=np.eye(4, dtype=np.float32))
    check_nn(lc, ids, d2, dst)


def test_icp_nn_zero_distance_ties():
    """Source points ON duplicated target points: d2 = 0 exactly, so the (d2, id) key the tile kernel
    minimises as an f64 is a denormal (just the id) — the lowest id must still win."""
    g = np.stack(np.meshgrid(np.arange(1, 9), np.arange(1, 9), np.arange(1, 4), indexing="ij"), -1).reshape(-1, 3)
    g = g.astype(np.float32) * np.float32(0.75) + np.float32(3.0)
    dst = np.concatenate([g, g[::-1], g]).astype(np.float32)  # every point three times, different ids
    src = np.ascontiguousarray(g[np.random.default_rng(2).permutation(len(g))])
    lc, r, ids, d2 = run(src, dst, 1.0, guess=np.eye(4, dtype=np.float32))
    check_nn(lc, ids, d2, dst)
    assert np.count_nonzero(d2 == 0) > len(src) // 2


def test_icp_nn_multi_iteration_prior():
    # a larger displacement: several ICP iterations, later passes seeded with the previous NN
    src, dst, _ = synth.make_icp_pair(n_points=20_000, seed=9, disp=(1.0, 4.0))
    lc, r, ids, d2 = run(src, dst, 1.0)
    assert r.iterations >= 2
    check_nn(lc, ids, d2, dst)


@pytest.mark.parametrize("n", [2, 4])
def test_icp_group_bit_identical_to_one_handle(n):
    """lio_icp_group (single-process multi-GPU): n ranks — all on device 0 on a one-GPU
    box, so the records travel through host memory; distinct devices use RCCL — give the one-handle
    transform, score, iterations and aligned cloud bit for bit."""
    src, dst, _ = synth.make_icp_pair(n_points=60_000, seed=12, disp=(1.0, 3.0))
    grp = LC.LoopClosureGroup(LC.LoopClosureConfig(), n, devices=[0] * n)
    assert not grp.uses_rccl
    grp.setInputSource(src)
    grp.setInputTarget(dst)
    rg = grp.align()
    one = LC.LoopClosure(LC.LoopClosureConfig())
    one.setInputSource(src)
    one.setInputTarget(dst)
    r1 = one.align()
    assert rg.iterations == r1.iterations >= 2 and rg.score == r1.score and rg.state == r1.state
    np.testing.assert_array_equal(np.array(list(rg.T)), np.array(list(r1.T)))
    np.testing.assert_array_equal(grp.aligned_, one.aligned_)


@pytest.mark.skipif(LC._capi.lib().lio_device_count() < 2, reason="RCCL exchange needs two distinct devices")
def test_icp_group_rccl_bit_identical():
    src, dst, _ = synth.make_icp_pair(n_points=60_000, seed=12, disp=(1.0, 3.0))
    grp = LC.LoopClosureGroup(LC.LoopClosureConfig(), 2)
    assert grp.uses_rccl
    grp.setInputSource(src)
    grp.setInputTarget(dst)
    rg = grp.align()
    one = LC.LoopClosure(LC.LoopClosureConfig())
    one.setInputSource(src)
    one.setInputTarget(dst)
    r1 = one.align()
    assert rg.iterations == r1.iterations and rg.score == r1.score
    np.testing.assert_array_equal(np.array(list(rg.T)), np.array(list(r1.T)))
