#!/bin/bash
# SQ counter passes over tools/kbbench (each pass its own run, <= 8 SQ counters).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
python - << 'PY'
import numpy as np
from fantoch_amd.workload import Workload
s = Workload.zipf(0.7, 1 << 20, k=1).generate(1_000_000)
s.keys[:, 0].astype(np.uint32).tofile("/tmp/kb_keys.u32")
s.dots.astype(np.uint64).tofile("/tmp/kb_dots.u64")
PY
OUT=gpurun_out/kbpmc
rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- tools/kbbench /tmp/kb_keys.u32 /tmp/kb_dots.u64 1000000 20 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python - << 'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/kbpmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "order" if "k_kb_order" in r["Kernel_Name"] else "partition" if "k_kb_partition" in r["Kernel_Name"] else None
        if k: agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
