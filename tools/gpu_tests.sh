#!/bin/bash
# The GPU suite (or $TESTS), one process, per-test timeouts; log in gpurun_out/.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --durations=12 --timeout 600 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -16 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_all.log | head -30; exit 1; }
