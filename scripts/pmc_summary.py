"""Fold the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of a bench run into
profiles/pmc_summary.json (read by bench.py for roofline.traffic).

HBM bytes per kNN h-evaluation = sum over its kernels (knn_near, knn_far,
plane) of 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes); the factor 2 is the
gfx950 FETCH_SIZE correction of /opt/skills/guides/MI355X_MICROARCH.md (HBM
section: FETCH_SIZE reports half the bytes of 16-B/lane reads).  Infinity-Cache
hits are counted by these counters (same section), so this is traffic leaving L2.
usage: python scripts/pmc_summary.py gpurun_out/<tag> C2 [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

src, cfg = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "profiles", "pmc_summary.json")
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
for name, d in per.items():
    short = name.split("(")[0].replace("void ", "").replace("lio::", "")
    kern[short] = {c: sum(v) / len(v) for c, v in d.items()}
    kern[short]["dispatches"] = max(len(v) for v in d.values())


def bytes_of(prefix):
    """per-dispatch bytes of the kernel(s) whose short name starts with prefix (template
    instantiations such as plane_kernel<2>, knn_far_kernel<false>), weighted by dispatches"""
    ks = [k for k in kern if k.split("<")[0] == prefix]
    n = sum(kern[k]["dispatches"] for k in ks)
    tot = sum(1024.0 * (2.0 * kern[k].get("FETCH_SIZE", 0.0) + kern[k].get("WRITE_SIZE", 0.0)) * kern[k]["dispatches"]
              for k in ks)
    return tot / max(n, 1)


# one near pass per kNN evaluation: its instantiations (first / seeded later evaluations) are
# averaged, weighted by their dispatch counts
total = sum(bytes_of(k) for k in ["knn_near_kernel", "knn_far_kernel", "plane_kernel"])
res = {"config": cfg, "knn_hbm_bytes_per_launch": round(total),
       "reuse_hbm_bytes_per_launch": round(bytes_of("h_model_reuse_kernel")),
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace only); "
                 "bytes = 1024*(2*FETCH_SIZE + WRITE_SIZE) per dispatch (gfx950 FETCH_SIZE x2 correction)",
       "kernels": {k: {c: round(v, 1) for c, v in d.items()} for k, d in sorted(kern.items())}}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("config", "knn_hbm_bytes_per_launch", "reuse_hbm_bytes_per_launch")}))
