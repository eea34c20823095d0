#!/bin/bash
# Streaming check: the executor / partial-executor GPU tests, the streaming
# tool (batches 1, 10, 1000) twice, and FH_GRAPH_DEBUG host + kernel phase
# times at batches of 1000 and 1.  One limit per step; stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-sc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_executor_gpu.py tests/test_partial_exec_gpu.py tests/test_execlog_gpu.py} -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { tail -30 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
rm -f $OUT/stream_$TAG.txt
for r in 1 2; do
  timeout -k 10 120 tools/stream_bench 1 20000 10 100000 1000 2000000 >> $OUT/stream_$TAG.txt 2>&1 || { cat $OUT/stream_$TAG.txt; exit 1; }
done
cat $OUT/stream_$TAG.txt
FH_GRAPH_DEBUG=1 timeout -k 10 60 tools/stream_bench 1000 20000 > /dev/null 2> $OUT/stream_dbg_$TAG.err || { tail -5 $OUT/stream_dbg_$TAG.err; exit 1; }
tail -6 $OUT/stream_dbg_$TAG.err
FH_GRAPH_DEBUG=1 timeout -k 10 60 tools/stream_bench 1 2000 > /dev/null 2> $OUT/stream_dbg1_$TAG.err || { tail -5 $OUT/stream_dbg1_$TAG.err; exit 1; }
tail -3 $OUT/stream_dbg1_$TAG.err
echo "== done"
