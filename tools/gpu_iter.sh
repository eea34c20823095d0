#!/bin/bash
# GPU iteration: selected parity tests, bench.py (args: extra bench flags),
# then a rocprofv3 kernel-trace summary of a short bench run.  Every GPU step
# has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TESTS=${TESTS:-tests/test_engine_gpu.py tests/test_fullsize_gpu.py}
TAG=${TAG:-iter}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?
  tail -4 $OUT/pytest_$TAG.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -40 $OUT/pytest_$TAG.log; exit $rc; fi
fi
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -30 $OUT/bench_$TAG.err; exit 1; }
python3 - $OUT/bench_$TAG.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
print("phases", d.get("phases_ms"))
print("kernels", {k: (round(v["avg_launch_us"], 1), v["launches"]) for k, v in d.get("kernels", {}).items()})
print("configs", {k: v["ms_per_step"] for k, v in d.get("configs", {}).items()})
PY
if [ -n "$NOPROF" ]; then exit 0; fi
rm -rf $OUT/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-phases --no-configs > $OUT/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -30 $OUT/prof_$TAG.log; exit 1; }
f=$(find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" $OUT/kernel_stats_$TAG.csv
python3 - "$OUT/kernel_stats_$TAG.csv" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    m = re.findall(r'(k_\w+|__amd\w+)(<[^>]*>)?', r["Name"])
    name = m[0][0] + (m[0][1] or '')[:40] if m else r["Name"][:60]
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {name}')
print(f"total {tot/1e6:.1f} ms")
PY
