#!/usr/bin/env python
"""Per-launch kernel durations from a rocprofv3 kernel-trace CSV, in launch
order, for the last step of a probe: the launches after the last
k_view_records (the step's first kernel), one line each (us), with runs of
the same kernel folded when short.

Usage: python tools/trace_launches.py run_kernel_trace.csv"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_view_records" in r["Kernel_Name"]]
    rows = rows[starts[-1]:] if starts else rows
    t0 = int(rows[0]["Start_Timestamp"])
    tot = {}
    for r in rows:
        n = short(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[n] = tot.get(n, 0.0) + d
        if d >= 50:
            print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:10.1f} {d:9.1f}  {n}")
    print("-- totals (us) --")
    for n, d in sorted(tot.items(), key=lambda x: -x[1])[:30]:
        print(f"{d:10.1f}  {n}")
    print(f"step span {(int(rows[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
