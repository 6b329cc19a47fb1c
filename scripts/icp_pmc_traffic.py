"""HBM traffic per ICP tile-kernel dispatch from separate rocprofv3 passes (FETCH_SIZE, WRITE_SIZE), with the
kernel durations of a --kernel-trace run of the same command (scripts/icp_ab.py 1.0 1: pair A then pair B).

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; the x2 is the gfx950 correction, MI355X_MICROARCH.md HBM
section).  Algorithmic bytes per pass: 500 k source points x 24 B = 12 MB, the figure rounds 2-3 used
(DESIGN §4 ICP row: this design's floor is ~3x that — tile points, current and prior correspondences,
writes and the 8 MB target).
usage: python scripts/icp_pmc_traffic.py <dir with icptrace/ icpfetch/ icpwrite/> <out.json>"""
import csv
import glob
import json
import os
import sys

KERNEL = "icp_tile_kernel"
ALG_BYTES = 12_000_000


def counters(d, name):
    vals = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(f)) if KERNEL in r.get("Kernel_Name", "") and r["Counter_Name"] == name]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
        vals += [float(r["Counter_Value"]) for r in rows]
    return vals


def durations(d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(f)) if KERNEL in r.get("Kernel_Name", "")]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
        out += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    return out


def main():
    base, dst = sys.argv[1], sys.argv[2]
    fetch = counters(os.path.join(base, "icpfetch"), "FETCH_SIZE")
    write = counters(os.path.join(base, "icpwrite"), "WRITE_SIZE")
    dur = durations(os.path.join(base, "icptrace"))
    n = min(len(fetch), len(write))
    passes = []
    for i in range(n):
        t = (2.0 * fetch[i] + write[i]) * 1024.0
        p = {"dispatch": i, "fetch_kib": fetch[i], "write_kib": write[i], "hbm_traffic_bytes": int(t),
             "x_algorithmic": round(t / ALG_BYTES, 2)}
        if i < len(dur):
            p["duration_us"] = round(dur[i], 1)
        passes.append(p)
    mean = sum(p["hbm_traffic_bytes"] for p in passes) / max(n, 1)
    res = {"kernel": KERNEL, "workload": "scripts/icp_ab.py 1.0 1 (C4 500k vs 500k; pair A then pair B, each a "
                                         "warm-up alignment then one timed one)",
           "method": "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs + a --kernel-trace run; "
                     "traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB)",
           "algorithmic_bytes_per_pass": ALG_BYTES, "dispatches": n,
           "mean_hbm_traffic_bytes": int(mean), "mean_x_algorithmic": round(mean / ALG_BYTES, 2),
           "max_x_algorithmic": max((p["x_algorithmic"] for p in passes), default=None),
           "passes": passes}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "passes"}))
    for p in passes:
        print(p)


if __name__ == "__main__":
    main()
