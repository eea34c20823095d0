cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "FH_VIEW_CMD=1" "FH_VIEW_CMD=1 FH_SRCH_DIAG=4" "FH_VIEW_CMD=1 FH_SRCH_DIAG=1"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-phases --probe view_search,view_records > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "$cfg failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],3), {k:(round(v['avg_launch_us'],1), v['launches']) for k,v in d['kernels'].items()})"
done
