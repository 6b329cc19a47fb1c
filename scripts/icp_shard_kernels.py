"""Per-rank kernel time of a sharded loop-ICP run from a rocprofv3 kernel trace (scripts/icp_shard_profile.py
under `rocprofv3 --kernel-trace`): every rank's kernels run on its own HIP stream, so the trace split by
Stream_Id gives each rank's per-pass kernel time — the split work (correspondences, records, compaction, the
window's chain blocks, depth blocks) against the redundant work (the event walk over all ranks' events, the
exchanges' merges, pcl_pack).

    python scripts/icp_shard_kernels.py <kernel_trace.csv> [out.txt]

Only streams that ran icp_tile_kernel are ranks; passes = that stream's tile launches (fitness passes included)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    by[r["Stream_Id"]].append(r)


def short(name):
    m = re.search(r"lio::(?:\(anonymous namespace\)::)?([A-Za-z0-9_]+)", name)
    if m:
        return m.group(1)
    return "copy" if "copyBuffer" in name else ("fill" if "fillBuffer" in name else name[:40])


lines = []
ranks = []
for sid, rs in sorted(by.items(), key=lambda kv: min(int(r["Start_Timestamp"]) for r in kv[1])):
    names = [short(r["Kernel_Name"]) for r in rs]
    if "icp_tile_kernel" not in names:
        continue
    passes = names.count("icp_tile_kernel")
    tot = collections.Counter()
    for r, nm in zip(rs, names):
        tot[nm] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ranks.append((sid, passes, tot))
for k, (sid, passes, tot) in enumerate(ranks):
    allk = sum(tot.values())
    lines.append(f"stream {sid} (rank {k}): {passes} passes, kernel time {allk / passes:.1f} us per pass")
    for nm, us in tot.most_common(14):
        lines.append(f"    {nm:32s} {us / passes:8.1f} us per pass")
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
