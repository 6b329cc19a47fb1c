"""The C++ C5 stream driver (tests/cpp/c5_stream.cpp) over the bench's eight sweeps, N times, with the
preprocess host phases on stderr (LIO_PREP_PROFILE=1): where the C++ preprocess stage's time goes.
usage: python scripts/cpp_stream_profile.py [runs]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))
from lio_gpu import pipeline as PL  # noqa: E402
from lio_gpu import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
mp, L, sp, kind = synth.CONFIGS["C5"]
scene = synth.make_scene(L, 1234)
m = synth.sample_surface(scene, mp, 1234)
stream = synth.make_loop_stream(scene, n_out=6, n_points=sp, kind=kind)
with tempfile.TemporaryDirectory() as td:
    fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
    PL.write_stream_input(fin, m, stream, synth.initial_cov(), 2)
    for r in range(runs):
        for ht in ("4", "8"):
            env = dict(os.environ, LIO_PREP_PROFILE="1", LIO_HOST_THREADS=ht)
            print(f"LIO_HOST_THREADS={ht}", flush=True)
            p = subprocess.run([PL.CPP_STREAM_EXE, fin, fout], capture_output=True, text=True, env=env, timeout=300)
            print(p.stdout.strip(), flush=True)
            errf = os.path.join(td, "err.txt")
            open(errf, "w").write(p.stderr)
            print(subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prep_profile_summary.py"), errf],
                                 capture_output=True, text=True).stdout, flush=True)
