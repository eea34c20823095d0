#!/bin/bash
# Diagnostic A/B on the C4 bench: each configuration (env assignments, space
# separated; CFGS overrides the list) runs a short C4-only bench and prints
# the step time and the probed kernels; FH_GRAPH_DEBUG lines are kept.
# Within one configuration, commas separate several assignments.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
PROBE=${PROBE:-sort_scatter_dots,graph_tile,cmd_search,view_records,cmd_pack,cmd_union}
i=0
for cfg in ${CFGS:-"X=0" "FH_SRCH_DIAG=1" "FH_SRCH_DIAG=2" "FH_SRCH_DIAG=4" "FH_SRCH_DIAG=6" "FH_GRAPH_DEBUG=1"}; do
  i=$((i+1))
  env ${cfg//,/ } timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-c5 --probe $PROBE > $OUT/diag_$i.json 2> $OUT/diag_$i.err || { echo "$cfg failed"; tail -20 $OUT/diag_$i.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$OUT/diag_$i.json').read().strip().splitlines()[-1])
print('$cfg', round(d['ms_per_step'], 3), {k: (round(v['avg_launch_us'], 1), v['launches']) for k, v in d['kernels'].items()})
print('   phases', {k: round(v, 2) for k, v in d.get('phases_ms', {}).items() if v > 0.05})
"
  grep "fh graph" $OUT/diag_$i.err | sort | uniq -c | head -8
done
