#!/bin/bash
# Graph-path session: engine/executor parity tests, then the config bench
# with graph iteration counters (FH_GRAPH_DEBUG).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_graph.log 2>&1
rc=$?
tail -3 $OUT/pytest_graph.log
if [ $rc -ne 0 ]; then tail -40 $OUT/pytest_graph.log; exit $rc; fi
FH_GRAPH_DEBUG=1 timeout -k 10 400 python -u tools/bench_configs.py --no-cpu ${CONFIGS_ARGS} > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -20 $OUT/configs.err; exit 1; }
grep "fh graph" $OUT/configs.err | sort | uniq -c | head -20
python - <<'PY'
import json
for l in open("gpurun_out/configs.jsonl"):
    d = json.loads(l)
    top = sorted(d["phases_ms"].items(), key=lambda x: -x[1])[:5]
    print(d["config"], "%.2f ms" % d["ms_per_step"], "%.3g cmds/s" % d["value"], top)
PY
