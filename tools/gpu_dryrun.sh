#!/bin/bash
# C5 fh_dgraph dry runs: N ranks sharing the box's one GPU over gloo (not a
# measurement of multi-GPU speed: the stages share one GPU and the exchanges
# go through host memory), for the condensed graph's size and the per-rank
# stage times at N stream ranges.  $NS: rank counts, one run each, each under
# its own time limit; stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-dry}
port=29511
for n in ${NS:-2 4}; do
  echo "== N=$n $(date +%T)"
  timeout -k 10 ${LIMIT:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --one-gpu --c5-backend gloo \
    --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-secondary --no-streaming --no-phases \
    --c5-steps 1 $DRY_ARGS > $OUT/dry_${TAG}_n$n.json 2> $OUT/dry_${TAG}_n$n.err || { tail -30 $OUT/dry_${TAG}_n$n.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['c5'];print(c['ms_per_step'],c['condensed_graph'],c['rank0_stage_ms'])" $OUT/dry_${TAG}_n$n.json
  port=$((port+1))
done
echo "== done $(date +%T)"
