#!/usr/bin/env python
"""Short table of a rocprofv3 kernel_stats.csv: kernel, calls, average us,
ms per step (steps = argv[2], default 13: 10 timed + 3 warmup)."""
import csv
import re
import sys

steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    m = re.search(r"(k_\w+|__amd\w+)(<[^(]*?>)?", n)
    short = (m.group(1) + (m.group(2) or "")) if m else n[:60]
    short = short.replace("fh::(anonymous namespace)::", "").replace("unsigned int", "u32")[:70]
    print(f"{short:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  "
          f"{float(r['TotalDurationNs'])/1e6/steps:7.3f} ms/step")
