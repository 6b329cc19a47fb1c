"""The host worker pool the uploads use (lio_pool.hpp): correctness with one and with several callers,
built with g++ and run plain and under ThreadSanitizer (host code only; no GPU)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpp", "test_host_pool.cpp")
INC = os.path.join(HERE, "..", "fast-lio-sam_gps_amd", "csrc")


@pytest.mark.parametrize("san", ["", "thread"])
def test_host_pool(tmp_path, san):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path / "pool")
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", "-I", INC, SRC, "-o", exe]
    if san:
        cmd.insert(1, f"-fsanitize={san}")
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0 bad2 0" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
