#!/bin/bash
# graph_tile certificate failures vs the first reach bound (C4 headline)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 256 384 512 768; do
  FH_TILE_R0=$r FH_GRAPH_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-phases > gpurun_out/r0_$r.json 2> gpurun_out/r0_$r.err || exit 1
  echo "== R0 first $r"; grep "graph_tile" gpurun_out/r0_$r.err | head -3
done
