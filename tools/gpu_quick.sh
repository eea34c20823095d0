#!/bin/bash
# Quick GPU iteration: selected parity tests, smoke, then bench.py with the
# given extra arguments.  Each GPU step has its own time limit; stops at the
# first crash / time limit.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TESTS=${TESTS:-tests/test_engine_gpu.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -q --durations=15 --timeout 400 --timeout-method thread > $OUT/pytest_q.log 2>&1
  rc=$?
  tail -15 $OUT/pytest_q.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
