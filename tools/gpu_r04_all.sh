#!/bin/bash
# Round-4 validation + measurement in one GPU call: $TESTS (default: the
# whole GPU suite), smoke, the C4-only bench line, the streaming tool and its
# kernel trace, and the C5 probe with the graph counters.  Every GPU step has
# its own limit; the script stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r04}
mkdir -p $OUT
if [ -n "$PRE_TESTS" ]; then
  echo "== pre-tests $(date +%T)"
  timeout -k 10 300 python -u -m pytest $PRE_TESTS -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_pre_$TAG.log 2>&1 || { tail -30 $OUT/pytest_pre_$TAG.log; exit 1; }
  tail -2 $OUT/pytest_pre_$TAG.log
fi
SMOKE=1 TESTS="${TESTS:-tests}" TAG=$TAG bash tools/gpu_r04.sh || exit 1
echo "== c4 bench $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-secondary --no-c5 --no-streaming > $OUT/bench_c4_$TAG.json 2> $OUT/bench_c4_$TAG.err || { tail -20 $OUT/bench_c4_$TAG.err; exit 1; }
echo "== streaming $(date +%T)"
timeout -k 10 120 tools/stream_bench 1 20000 10 100000 1000 2000000 > $OUT/stream_$TAG.txt 2>&1 || { cat $OUT/stream_$TAG.txt; exit 1; }
cat $OUT/stream_$TAG.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sbprof_$TAG -o sb -- tools/stream_bench 1 5000 1000 1000000 > $OUT/sbprof_$TAG.log 2>&1 || { tail -20 $OUT/sbprof_$TAG.log; exit 1; }
FH_GRAPH_DEBUG=1 timeout -k 10 60 tools/stream_bench 1000 20000 > $OUT/stream_dbg_$TAG.txt 2> $OUT/stream_dbg_$TAG.err || { tail -5 $OUT/stream_dbg_$TAG.err; exit 1; }
tail -3 $OUT/stream_dbg_$TAG.err
echo "== c5 probe $(date +%T)"
FH_GRAPH_DEBUG=1 timeout -k 10 300 python -u tools/c5_probe.py --steps 2 > $OUT/c5dbg_$TAG.log 2>&1 || { tail -20 $OUT/c5dbg_$TAG.log; exit 1; }
grep -v "^\[W" $OUT/c5dbg_$TAG.log | tail -4
echo "== done $(date +%T)"
