"""icp_tile_kernel duration per launch (us) from a rocprofv3 kernel trace, in launch order, with the mean
(scripts/icp_ab.py 1.0 1 under `rocprofv3 --kernel-trace`: pair A x3 alignments, then pair B x3).

    python scripts/icp_tile_passes.py <kernel_trace.csv> [label]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "icp_tile_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
label = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"# icp_tile_kernel duration per pass (us) {label}")
print(" ".join(f"{x:.1f}" for x in d))
print(f"mean {sum(d) / max(len(d), 1):.1f}  launches {len(d)}")
