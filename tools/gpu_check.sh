#!/bin/bash
# One GPU-box session: parity suite (-m gpu), smoke, bench, kernel-trace stats.
# Every GPU step has its own time limit.  A test FAILURE (exit 1) still lets
# the bench run; a crash, abort, fault or time limit ends the script there.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -n "$QUICK" ]; then exit $rc; fi
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-phases > $OUT/prof.log 2>&1 || { echo rocprof failed; tail -30 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $OUT/kernel_stats_$TAG.csv
head -12 $OUT/kernel_stats_$TAG.csv | cut -c1-220
exit $rc
