#!/bin/bash
# rocprofv3 kernel-trace summary of tools/bench_configs.py for one config
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
CFG=${CFG:-c5}
TAG=${TAG:-prof_$CFG}
rm -rf $OUT/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$TAG -o run -- python3 tools/bench_configs.py --only $CFG --no-cpu --steps 2 > $OUT/$TAG.log 2>&1 || { echo rocprof failed; tail -20 $OUT/$TAG.log; exit 1; }
f=$(find $OUT/$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" $OUT/kernel_stats_$TAG.csv
python3 - "$OUT/kernel_stats_$TAG.csv" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:30]:
    m = re.findall(r'(k_\w+|__amd\w+)(<[^>]*>)?', r["Name"])
    name = m[0][0] + (m[0][1] or '') if m else r["Name"][:60]
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {name}')
print(f"total {tot/1e6:.1f} ms")
PY
