#!/bin/bash
# graph_tile on the C4 headline: FH_GRAPH_DEBUG stats of a warm run + bench
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
FH_GRAPH_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/ab_dbg.json 2> $OUT/ab_dbg.err || exit 1
grep "graph_tile" $OUT/ab_dbg.err | tail -4
