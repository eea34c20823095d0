#!/bin/bash
# Round-6 probes: the C4 key shard (tools/shard_probe.py) and the C2 line
# (tools/c2_phases.py), each as a plain run, then under rocprofv3 kernel
# stats.  Every GPU step has its own time limit; stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r06p}
mkdir -p $OUT
step() { echo "== $1 $(date +%T)"; }
rm -rf $OUT/prof_shard_$TAG $OUT/prof_c2_$TAG
step shard
timeout -k 10 300 python -u tools/shard_probe.py > $OUT/shard_$TAG.json 2> $OUT/shard_$TAG.err || { tail -20 $OUT/shard_$TAG.err; exit 1; }
cat $OUT/shard_$TAG.json
step shard_debug
FH_GRAPH_DEBUG=1 timeout -k 10 300 python -u tools/shard_probe.py > $OUT/shard_dbg_$TAG.json 2> $OUT/shard_dbg_$TAG.err || { tail -20 $OUT/shard_dbg_$TAG.err; exit 1; }
grep phases $OUT/shard_dbg_$TAG.err | tail -2
step shard_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard_$TAG -o run -- python3 tools/shard_probe.py > $OUT/prof_shard_$TAG.log 2>&1 || { tail -20 $OUT/prof_shard_$TAG.log; exit 1; }
find $OUT/prof_shard_$TAG -name '*kernel_trace.csv' -delete
step c2
timeout -k 10 300 python -u tools/c2_phases.py > $OUT/c2_$TAG.txt 2>&1 || { tail -20 $OUT/c2_$TAG.txt; exit 1; }
cat $OUT/c2_$TAG.txt | tail -20
step c2_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2_$TAG -o run -- python3 tools/c2_phases.py > $OUT/prof_c2_$TAG.log 2>&1 || { tail -20 $OUT/prof_c2_$TAG.log; exit 1; }
find $OUT/prof_c2_$TAG -name '*kernel_trace.csv' -delete
step done
