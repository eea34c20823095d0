#!/bin/bash
# C4 iteration: smoke, then a C4-only bench line with phases and kernel probes.
# Optional: TESTS="<pytest paths>" runs those GPU tests first; CFGS="A=1 B=2 ..."
# (space-separated env assignments, ';' between configurations) A/Bs the bench.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --durations=10 --timeout 400 --timeout-method thread > $OUT/pytest_c4.log 2>&1
  rc=$?; tail -12 $OUT/pytest_c4.log; [ $rc -eq 0 ] || { tail -60 $OUT/pytest_c4.log; exit 1; }
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
C4="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs --no-c5 $BENCH_ARGS"
IFS=';' read -ra CONFS <<< "${CFGS:-FH_X=0}"
i=0
for cfg in "${CONFS[@]}"; do
  env $cfg timeout -k 10 300 python -u $C4 > $OUT/c4_$i.json 2> $OUT/c4_$i.err || { tail -30 $OUT/c4_$i.err; exit 1; }
  python -c "
import json;d=json.loads(open('$OUT/c4_$i.json').read().strip().splitlines()[-1])
print('[$cfg]', round(d['ms_per_step'],3), 'cold', d['cold_ms'])
print(' phases', {k:v for k,v in d.get('phases_ms',{}).items() if v>0.05})
print(' kernels', {k:(round(v['avg_launch_us'],1), v['launches']) for k,v in d['kernels'].items()})"
  i=$((i+1))
done
