cd /root/repo
for c in 3000000 6000000 12582912 25000000; do
  echo "chunk $c"
  FH_VIEW_CHUNK=$c timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/sw_$c.json 2>gpurun_out/sw_$c.err || { tail -5 gpurun_out/sw_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw_$c.json')); print(d['ms_per_step'], d['phases_ms'].get('keydeps_views'), d['phases_ms'].get('graph_tile'))"
done
