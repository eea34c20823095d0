#!/bin/bash
# C2 (single view) parity tests, then the secondary bench line under a kernel
# trace: k_kb_step average per 1M-command batch.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_keydeps_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "c2 or keydeps or single or noops or batches" > $OUT/pytest_c2.log 2>&1; rc=$?
tail -3 $OUT/pytest_c2.log
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_c2.log; exit $rc; }
rm -rf $OUT/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 -c "
import sys; sys.path.insert(0, '.')
import bench
class A: pass
r = bench.secondary_c2(A(), 0)
print(r['ms_per_step'])
" > $OUT/prof_c2.log 2>&1 || { tail -20 $OUT/prof_c2.log; exit 1; }
tail -2 $OUT/prof_c2.log
f=$(find $OUT/prof_c2 -name '*kernel_stats.csv' | head -1)
grep -E "kb_step|kb_partition|kb_order" "$f" | cut -c1-200
