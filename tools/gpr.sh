#!/bin/bash
# gpurun with retries on transient pool failures only (no box / box not ready /
# back-off: nothing ran, nothing charged).  Usage: tools/gpr.sh <timeout> <out> <command>
T=$1; OUT=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $OUT 2>&1
  grep -q "status=transient" $OUT || break
  w=$(grep -o "retry in [0-9]*s" $OUT | grep -o "[0-9]*" | head -1)
  sleep $(( ${w:-60} + 10 ))
done
cat $OUT
