#!/bin/bash
# Round-3 GPU batch: the partial-replication lock-step tests, multi-engine
# staging, the streaming benchmark of fh_graph at batch 1 / 1k / 1M, and the
# tile kernel's phase profile on C4.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_partial_exec_gpu.py tests/test_multi_gpu.py tests/test_executor_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_b.log 2>&1
rc=$?; tail -25 $OUT/pytest_b.log; [ $rc -eq 0 ] || exit 1
echo "== stream_bench $(date +%T)"
timeout -k 10 400 tools/stream_bench 1 20000 1000 2000000 1000000 20000000 > $OUT/stream_bench.json 2> $OUT/stream_bench.err || { cat $OUT/stream_bench.err; exit 1; }
cat $OUT/stream_bench.json
echo "== tile phases $(date +%T)"
FH_GRAPH_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-configs --no-c5 --no-phases > $OUT/tile_dbg.json 2> $OUT/tile_dbg.err || { tail -20 $OUT/tile_dbg.err; exit 1; }
grep "fh graph" $OUT/tile_dbg.err | tail -8
echo "== done $(date +%T)"
