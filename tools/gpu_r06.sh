#!/bin/bash
# Round-6 GPU session: $TESTS (pytest node ids, default none), then the C4
# bench sweep ($SWEEP entries, tools/gpu_sweep.sh), then optionally the
# C4-only rocprofv3 stats ($PROF=1).  Every GPU step has its own time limit;
# the script stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r06}
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TESTS" ]; then
  step pytest
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu -x -v --durations=10 --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest_gpu_$TAG.log | head -30; exit 1; }
fi
if [ -n "$SWEEP" ]; then
  TAG=$TAG bash tools/gpu_sweep.sh || exit 1
fi
if [ -n "$PROF" ]; then
  TAG=$TAG bash tools/gpu_r05_prof.sh || exit 1
fi
step done
