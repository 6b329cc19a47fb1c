"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code only).

`make -C oracle san` compiles oracle/san_driver.cpp (which includes the
oracle's translation unit) with -fsanitize=address,undefined and runs every
entry point once on the edge cases the parity tests use: empty and 1-point
maps, k = 1..8, ICP with no overlap and a 1-point target, deleting the whole
incremental map, VoxelGrid / submap / preprocess.  A sanitizer report fails the
run (-fno-sanitize-recover).  The checker has to be clean before its answers
can pin the GPU path.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")
def test_oracle_clean_under_asan_ubsan():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "san_driver: ok" in r.stdout
