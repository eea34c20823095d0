#!/bin/bash
# Streaming benchmark of fh_graph (batch 1 / 1k / 1M) and its kernel profile.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_partial_exec_gpu.py tests/test_executor_gpu.py tests/test_execlog_gpu.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_c.log 2>&1
rc=$?; tail -3 $OUT/pytest_c.log; [ $rc -eq 0 ] || { tail -30 $OUT/pytest_c.log; exit 1; }
echo "== stream_bench $(date +%T)"
timeout -k 10 400 tools/stream_bench 1 20000 1000 2000000 1000000 20000000 > $OUT/stream_bench.json 2> $OUT/stream_bench.err || { cat $OUT/stream_bench.err; exit 1; }
cat $OUT/stream_bench.json
rm -rf $OUT/prof_stream1 $OUT/prof_stream1m
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stream1 -o run -- tools/stream_bench 1 3000 > $OUT/prof_stream1.log 2>&1 || { tail -20 $OUT/prof_stream1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stream1m -o run -- tools/stream_bench 1000000 5000000 > $OUT/prof_stream1m.log 2>&1 || { tail -20 $OUT/prof_stream1m.log; exit 1; }
grep commands $OUT/prof_stream1.log $OUT/prof_stream1m.log
echo "== done $(date +%T)"
