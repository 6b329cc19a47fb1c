"""CPU checks of the C-ABI library: it loads, exports every symbol that
include/lio_gpu.h declares, its host-only helpers work, and its compute entry
points fail loudly (LIO_ERR_NODEV) when no gfx950 device is visible."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from lio_gpu import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "lio_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = "\n".join(line for line in src.splitlines() if not line.lstrip().startswith("typedef"))
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s+\*?([A-Za-z_][A-Za-z0-9_]*)\s*\(",
                       src, flags=re.M)
    return sorted(set(n for n in names if n not in ("typedef",)))


def test_header_declares_expected_api():
    fns = _header_functions()
    assert set(fns) == set(_capi.EXPORTS), set(fns) ^ set(_capi.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _capi.lib()
    for name in _header_functions():
        assert hasattr(L, name), name
    assert b"gfx950" in L.lio_build_info()


def test_exports_visible_to_nm():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in _header_functions() if n not in syms]
    assert not missing, missing


def test_host_only_shard_helpers():
    from lio_gpu import dist

    ns = 500_000
    for world in (1, 2, 3, 4, 8):
        spans = [dist.shard_range(ns, r, world) for r in range(world)]
        assert spans[0][0] == 0 and sum(n for _, n in spans) == ns
        for (b0, n0), (b1, _) in zip(spans, spans[1:]):
            assert b0 + n0 == b1 and b1 % 4096 == 0
    # combine = record-order sum of the slots
    rng = np.random.default_rng(0)
    nrec = (ns + 4095) // 4096
    recs = rng.normal(size=(nrec, 20))
    for world in (1, 2, 4, 8):
        slot = -(-nrec // world)
        recv = np.zeros((world, slot, 20))
        for r in range(world):
            s0, s1 = nrec * r // world, nrec * (r + 1) // world
            recv[r, : s1 - s0] = recs[s0:s1]
        out = dist.combine(recv.ravel(), ns, world)
        ref = np.zeros(17)
        for k in range(nrec):
            ref += recs[k, :17]
        np.testing.assert_array_equal(out, ref)


def test_compute_fails_loudly_without_device():
    L = _capi.lib()
    if L.lio_device_count() > 0:
        pytest.skip("a device is visible; covered by the gpu tests")
    h = C.c_void_p()
    rc = L.lio_map_create(C.byref(_capi.MapParams(1.0, 0.5, 0, 0)), C.byref(h))
    assert rc == _capi.LIO_ERR_NODEV and not h.value
    assert b"no HIP device" in L.lio_last_error() or b"gfx950" in L.lio_last_error()
    rc = L.lio_icp_create(C.byref(_capi.IcpParams(52.5, 0.01, 0.01, 50, 0.0, 1.5, 1.0, 0)), C.byref(h))
    assert rc == _capi.LIO_ERR_NODEV
    # the multi-GPU group and the one-shot icp_align(n_gpus) fail the same way (no CPU path)
    rc = L.lio_icp_group_create(C.byref(_capi.IcpParams(52.5, 0.01, 0.01, 50, 0.0, 1.5, 1.0, 0)), 2, None,
                                C.byref(h))
    assert rc == _capi.LIO_ERR_NODEV and not h.value
    pts = np.zeros((8, 3), np.float32)
    fp = pts.ctypes.data_as(C.POINTER(C.c_float))
    T = (C.c_float * 16)()
    rc = L.icp_align(fp, 8, fp, 8, C.byref(_capi.IcpParams(52.5, 0.01, 0.01, 50, 0.0, 1.5, 1.0, 0)), 4, T, None,
                     None, None, None)
    assert rc == _capi.LIO_ERR_NODEV


def _rot(axis, ang):
    a = np.asarray(axis, np.float64) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_icp_umeyama_pcl_float_host(seed):
    """Host half of the PCL-order fidelity mode (float JacobiSVD, lio_icp_umeyama_pcl_float): the sums
    the GPU returns (sequential float sums over the pairs) -> the rigid transform.  Checked against the
    known motion and numpy's double SVD Umeyama on the same pairs: within 1e-5 (float)."""
    rng = np.random.default_rng(seed)
    n = 2000
    src = (rng.standard_normal((n, 3)) * [8.0, 5.0, 1.5] + [30.0, -12.0, 2.0]).astype(np.float32)
    R = _rot(rng.standard_normal(3), rng.uniform(0.01, 0.3))
    t = rng.uniform(-2, 2, 3)
    tgt = (src.astype(np.float64) @ R.T + t + rng.standard_normal((n, 3)) * 0.01).astype(np.float32)
    sums = np.zeros(16, np.float32)
    sums[0:3] = np.cumsum(src, axis=0, dtype=np.float32)[-1]  # sequential float sums, Eigen's redux order
    sums[3:6] = np.cumsum(tgt, axis=0, dtype=np.float32)[-1]
    sums[6] = np.array([n], np.uint32).view(np.float32)[0]
    inv = np.float32(1.0) / np.float32(n)
    sm, dm = sums[0:3] * inv, sums[3:6] * inv
    prod = (tgt - dm)[:, :, None] * (src - sm)[:, None, :]  # float32 products, row r target, col c source
    sums[7:16] = np.cumsum(prod.reshape(n, 9), axis=0, dtype=np.float32)[-1]
    T = np.zeros(16, np.float32)
    L = _capi.lib()
    assert L.lio_icp_umeyama_pcl_float(sums.ctypes.data_as(_capi.fp), T.ctypes.data_as(_capi.fp)) == 0
    T = T.reshape(4, 4).astype(np.float64)
    # numpy double Umeyama on the same pairs
    s64, d64 = src.astype(np.float64), tgt.astype(np.float64)
    ms, md = s64.mean(0), d64.mean(0)
    U, _, Vt = np.linalg.svd((d64 - md).T @ (s64 - ms) / n)
    S = np.diag([1, 1, np.sign(np.linalg.det(U) * np.linalg.det(Vt))])
    Rn = U @ S @ Vt
    tn = md - Rn @ ms
    assert np.abs(T[:3, :3] - Rn).max() < 1e-5 and np.abs(T[:3, 3] - tn).max() < 2e-4
    assert np.abs(T[:3, :3] - R).max() < 1e-3
    assert np.abs(T[3] - [0, 0, 0, 1]).max() == 0
    assert abs(np.linalg.det(T[:3, :3]) - 1) < 1e-5


def test_abi_struct_sizes_match_the_binding(monkeypatch):
    """The round-4 segfault: an A/B of a round-2 build through LIO_GPU_LIB wrote its
    128-byte lio_kernel_timing (an extra finalize pair) into HEAD's 112-byte ctypes struct — a heap overrun
    that crashed the interpreter at exit.  The binding now compares every public struct's size with the
    library's (lio_abi_struct_sizes) at load and refuses a mismatch."""
    L = _capi.lib()
    n = L.lio_abi_struct_sizes(None, 0)
    sizes = (C.c_int64 * n)()
    L.lio_abi_struct_sizes(sizes, n)
    assert list(sizes) == [C.sizeof(getattr(_capi, k)) for k in _capi._ABI_STRUCTS]
    _capi._check_abi(L)  # HEAD against HEAD: accepted

    class RoundTwoTiming(C.Structure):  # the round-2 layout: one (launches, ms) pair more
        _fields_ = _capi.KernelTiming._fields_ + [("final_launches", C.c_int64), ("final_ms", C.c_double)]

    monkeypatch.setattr(_capi, "KernelTiming", RoundTwoTiming)
    with pytest.raises(ImportError, match="ABI mismatch"):
        _capi._check_abi(L)
