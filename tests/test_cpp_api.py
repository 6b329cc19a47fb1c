"""The C++ host-side mirror (include/lio_gpu.hpp) — what a FAST-LIO-SAM C++
maintainer links against: compiled with g++ against liblio_gpu.so here (CPU),
and run on the GPU (tests/cpp/test_cpp_api.cpp checks kNN bit-exact against a
brute-force scan, the IESKF pose recovery, map_incremental and icpAlignment)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "fast-lio-sam_gps_amd", "lio_gpu", "_lib")
SRC = os.path.join(ROOT, "tests", "cpp", "test_cpp_api.cpp")


def _build(tmp_path):
    exe = str(tmp_path / "test_cpp_api")
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
           "-L", LIBDIR, "-llio_gpu", "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def test_cpp_api_compiles_and_links(tmp_path):
    assert os.path.exists(os.path.join(LIBDIR, "liblio_gpu.so")), "build the library first (make -C fast-lio-sam_gps_amd)"
    _build(tmp_path)


@pytest.mark.gpu
def test_cpp_api_runs_on_gpu(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:])
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]
