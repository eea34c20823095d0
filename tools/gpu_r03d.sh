#!/bin/bash
# Round-3 GPU batch: the whole GPU suite (balanced radix digits and the
# register-cached tile sweeps touch every sort and the tile kernel), the
# balanced-vs-8-bit A/B on the C4 bench, fh_graph streaming, C5 profile.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
C4="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs --no-c5"
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 600 --timeout-method thread > $OUT/pytest_d.log 2>&1
rc=$?; tail -14 $OUT/pytest_d.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest_d.log; exit 1; }
echo "== A/B $(date +%T)"
ab() {  # ab <tag> <env...>: one C4 bench run under the given environment
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u $C4 > $OUT/ab_$tag.json 2> $OUT/ab_$tag.err || { tail -20 $OUT/ab_$tag.err; return 1; }
  python -c "import json;d=json.loads(open('$OUT/ab_$tag.json').read().strip().splitlines()[-1]);print('$tag', round(d['ms_per_step'],3), {k:v for k,v in d['phases_ms'].items() if v>0.1})"
}
ab base FH_X=0 && ab bal0 FH_SORT_BALANCED=0 && ab uc10 FH_UNION_CHUNK=10000000 && \
  ab uc10nt FH_UNION_CHUNK=10000000 FH_UNION_NT=1 && ab nt FH_UNION_NT=1 && ab uc5nt FH_UNION_CHUNK=5000000 FH_UNION_NT=1 || exit 1
echo "== stream_bench $(date +%T)"
timeout -k 10 400 tools/stream_bench 1 20000 1000 2000000 1000000 20000000 > $OUT/stream_bench.json 2> $OUT/stream_bench.err || { cat $OUT/stream_bench.err; exit 1; }
cat $OUT/stream_bench.json
rm -rf $OUT/prof_stream1 $OUT/prof_stream1m $OUT/prof_c5_r03
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stream1 -o run -- tools/stream_bench 1 3000 > $OUT/prof_stream1.log 2>&1 || { tail -20 $OUT/prof_stream1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stream1m -o run -- tools/stream_bench 1000000 5000000 > $OUT/prof_stream1m.log 2>&1 || { tail -20 $OUT/prof_stream1m.log; exit 1; }
echo "== c5 profile $(date +%T)"
FH_GRAPH_DEBUG=1 timeout -k 10 300 python -u tools/c5_probe.py --n 25000000 --steps 2 > $OUT/c5dbg.log 2> $OUT/c5dbg.err || { tail -20 $OUT/c5dbg.err; exit 1; }
grep "fh graph" $OUT/c5dbg.err | tail -4; tail -2 $OUT/c5dbg.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_r03 -o run -- python3 tools/c5_probe.py --n 25000000 --steps 2 > $OUT/prof_c5_r03.log 2>&1 || { tail -20 $OUT/prof_c5_r03.log; exit 1; }
# keep the summaries, drop the per-dispatch traces (gpurun_out/ travels back
# only under 64 MiB)
find $OUT -name '*kernel_trace.csv' -delete
echo "== done $(date +%T)"
