#!/usr/bin/env python3
"""Short per-kernel table from a rocprofv3 *_kernel_stats.csv: calls, average and total microseconds."""
import csv
import re
import sys

for f in sys.argv[1:]:
    print("==", f)
    for x in csv.DictReader(open(f)):
        n = x["Name"]
        m = re.search(r"(\w+_kernel|\w+kernel\w*)", n)
        short = (m.group(1) if m else n)[:48]
        if "rocprim" in n:
            short = "rocprim:" + (re.search(r"detail::(\w+)", n).group(1) if "detail::" in n else "")[:40]
        print(f'{short:50s} {x["Calls"]:>6} {float(x["AverageNs"]) / 1e3:9.2f} {float(x["TotalDurationNs"]) / 1e3:11.1f}')
