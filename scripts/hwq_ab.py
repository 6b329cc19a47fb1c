"""bench.py's multi_stream section (1, 2, 4, 8 independent scan streams on one GPU) under HIP's default 4
hardware queues per process and under GPU_MAX_HW_QUEUES = 8 / 16: does the stream count outrun the
hardware queues (streams sharing a queue run their kernels in turn)?"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for q in ("4", "8", "16"):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "5", "--no-cpu",
                        "--no-icp", "--pipeline", "0", "--streams", "1,2,4,8"], capture_output=True, text=True,
                       env=env, timeout=400)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    if p.returncode != 0 or not lines:
        print(f"GPU_MAX_HW_QUEUES={q}: bench failed rc={p.returncode}: {p.stderr[-500:]}", flush=True)
        sys.exit(1)
    d = json.loads(lines[-1])
    print(f"GPU_MAX_HW_QUEUES={q}: headline {d['value']} scans/s, multi_stream "
          f"{[(m['streams'], m['scans_per_s']) for m in d['multi_stream']]}", flush=True)
