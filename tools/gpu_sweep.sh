#!/bin/bash
# C4-only bench lines under several environment settings ($SWEEP: entries
# separated by ';', each a space-separated list of VAR=value, "-" for none).
# One bench process per entry, each under its own time limit; stops at the
# first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-sweep}
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-secondary --no-c5 --no-streaming}
IFS=';' read -ra ENTRIES <<< "$SWEEP"
i=0
for e in "${ENTRIES[@]}"; do
  [ "$e" = "-" ] && e=""
  echo "== [$e] $(date +%T)"
  env $e timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py $ARGS > $OUT/sweep_${TAG}_$i.json 2> $OUT/sweep_${TAG}_$i.err || { tail -20 $OUT/sweep_${TAG}_$i.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'], d.get('phases_ms'))" $OUT/sweep_${TAG}_$i.json
  i=$((i+1))
done
echo "== done $(date +%T)"
