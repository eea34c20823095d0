cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"X=0" "FH_SORT_WIDE=1" "FH_VIEW_CHUNK=12000000" "FH_VIEW_CHUNK=16500000"}; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-configs --no-phases > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "$cfg failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],3), {k:(round(v['avg_launch_us'],1), v['launches']) for k,v in d['kernels'].items()})"
done
