#!/bin/bash
# C5 probe under rocprofv3 --kernel-trace: the per-launch durations of the
# global path's kernels in launch order (tools/trace_launches.py), for the
# last step.  One GPU step, its own time limit.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-c5t}
rm -rf $OUT/prof_c5t_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c5t_$TAG -o run -- python3 tools/c5_probe.py --steps 2 > $OUT/prof_c5t_$TAG.log 2>&1 || { tail -20 $OUT/prof_c5t_$TAG.log; exit 1; }
f=$(find $OUT/prof_c5t_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_launches.py "$f" > $OUT/c5_launches_$TAG.txt
find $OUT/prof_c5t_$TAG -name '*kernel_trace.csv' -delete
tail -80 $OUT/c5_launches_$TAG.txt
