"""Medians of the LIO_PREP_PROFILE=1 lines (lio_scan_preprocess host phases) in a stderr capture.
usage: python scripts/prep_profile_summary.py <stderr file>"""
import collections
import statistics
import sys

vals = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    if not ln.startswith("prep_profile"):
        continue
    tok = ln.split()[1:]
    for k, v in zip(tok[0::2], tok[1::2]):
        try:
            vals[k].append(float(v))
        except ValueError:
            pass
print(" ".join(f"{k} p50 {statistics.median(v):.1f}" for k, v in vals.items() if k not in ("attempt",)))
att = vals.get("attempt", [])
print(f"calls {len(vals.get('total_us', []))} wait lines {len(att)} redo (attempt > 0) {sum(1 for a in att if a > 0)}")
