cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tile.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_tile.log; exit $rc; }
for cfg in "FH_TILE_MIXED=0" "FH_TILE_MIXED=1"; do
  env $cfg FH_GRAPH_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-phases --probe graph_tile > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "$cfg failed"; tail -5 gpurun_out/ab.err; exit 1; }
  grep "graph_tile mixed\|graph_tile: V" gpurun_out/ab.err | tail -2
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],3), {k:(round(v['avg_launch_us'],1), v['launches']) for k,v in d['kernels'].items()})"
done
