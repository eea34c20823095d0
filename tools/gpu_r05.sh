#!/bin/bash
# Round-5 GPU session: $TESTS (default the whole GPU suite), then optionally
# smoke and a bench line ($BENCH_ARGS).  Every GPU step has its own time limit;
# the script stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r05}
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 ${TEST_LIMIT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --durations=20 --timeout 600 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -28 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest_gpu_$TAG.log | head -30; exit 1; }
fi
if [ -n "$SMOKE" ]; then
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { cat $OUT/smoke_$TAG.log; exit 1; }
  cat $OUT/smoke_$TAG.log
fi
if [ -n "$BENCH" ]; then
  step bench
  timeout -k 10 ${BENCH_LIMIT:-600} python -u bench.py $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
step done
