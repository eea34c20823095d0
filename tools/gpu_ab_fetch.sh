#!/bin/bash
# Graph parity tests, then the config bench with the mailbox read-back (0)
# and with hipMemcpyAsync + hipStreamSynchronize (1), FH_GRAPH_DEBUG counters.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_executor_gpu.py tests/test_pred_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for m in ${MODES:-0 1}; do
  FH_FETCH_MEMCPY=$m FH_GRAPH_DEBUG=1 timeout -k 10 300 python tools/bench_configs.py --no-cpu ${CONFIGS_ARGS} > $OUT/c$m.jsonl 2> $OUT/c$m.err || { tail -20 $OUT/c$m.err; exit 1; }
  grep "fh graph" $OUT/c$m.err | sort | uniq -c | tail -6
  python - $OUT/c$m.jsonl $m <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    top = sorted(d["phases_ms"].items(), key=lambda x: -x[1])[:4]
    print("memcpy=%s" % sys.argv[2], d["config"], round(d["ms_per_step"], 2), top)
PY
done
