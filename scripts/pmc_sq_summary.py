"""Issue / wait breakdown of the hot kernels from one rocprofv3 --pmc pass of SQ + GRBM counters
(VERDICT r03 #5).  Per kernel (mean per dispatch):

  valu_busy_frac = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction issues over 2 cycles on a SIMD-32,
                   MI355X_MICROARCH.md "Per-instruction cycle constants") / (1024 SIMDs x kernel cycles), kernel
                   cycles = duration x 2.4 GHz for dispatches under 0.3 ms (the guide: GRBM_GUI_ACTIVE / 8 /
                   duration "reads high on dispatches shorter than about 0.3 ms"), else x that effective clock
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (waves parked on s_waitcnt / barriers: memory latency)
  issue_stall    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (ready but not issued: pipe / dependency stalls)
  active_frac    = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (the three are disjoint and sum to ~1, same guide)

usage: python scripts/pmc_sq_summary.py gpurun_out/<tag>/<pass dir> [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None
cnt = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        cnt[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
dur = {}
for f in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        dur[d] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9  # s
per = collections.defaultdict(list)
for d, c in cnt.items():
    k = names[d].split("(")[0].replace("void ", "").replace("lio::", "")
    if d in dur and dur[d] > 0:
        c = dict(c)
        c["_dur_s"] = dur[d]
        per[k].append(c)
res = {}
for k, lst in per.items():
    m = {c: sum(x.get(c, 0.0) for x in lst) / len(lst) for c in lst[0]}
    wc = m.get("SQ_WAVE_CYCLES", 0.0)
    grbm = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / m["_dur_s"] if m.get("GRBM_GUI_ACTIVE") else None
    clock = grbm if (grbm and m["_dur_s"] >= 3e-4) else 2.4e9
    cyc = m["_dur_s"] * clock
    res[k] = {"dispatches": len(lst), "avg_us": round(m["_dur_s"] * 1e6, 2), "clock_ghz": round(clock / 1e9, 3),
              "grbm_clock_ghz": round(grbm / 1e9, 3) if grbm else None,
              "valu_insts": round(m.get("SQ_INSTS_VALU", 0.0)),
              "valu_busy_frac": round(m.get("SQ_INSTS_VALU", 0.0) * 2.0 / (1024.0 * cyc), 4) if cyc else None,
              "wait_frac": round(m.get("SQ_WAIT_ANY", 0.0) / wc, 4) if wc else None,
              "issue_stall_frac": round(m.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4) if wc else None,
              "active_frac": round(m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4) if wc else None}
for k in sorted(res, key=lambda k: -res[k]["avg_us"] * res[k]["dispatches"])[:20]:
    print(f"{k[:60]:60s} {json.dumps(res[k])}")
if out:
    json.dump(res, open(out, "w"), indent=1)
