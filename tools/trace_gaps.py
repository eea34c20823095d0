"""Print kernel durations and gaps from a rocprofv3 kernel trace (per queue)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 16
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:first + count]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void fh::(anonymous namespace)::", "")[:28]
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"q{q:>3} {name:28s} start +{(st - t0) / 1000:8.2f} us  dur {(en - st) / 1000:7.2f} us")
