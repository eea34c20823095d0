#!/bin/bash
# One GPU-box session: parity suite, smoke, bench, kernel-trace stats, and the
# four PMC passes of tools/collect_pmc.py.  Every GPU step has its own time
# limit and the steps are chained: the script stops at the first failure.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-phases"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
cat $OUT/bench.json
rm -rf $OUT/prof $OUT/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $BENCH > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python3 $BENCH > $OUT/pmc_fetch.log 2>&1 || { tail -30 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python3 $BENCH > $OUT/pmc_write.log 2>&1 || { tail -30 $OUT/pmc_write.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/calib_fetch -o run -- tools/pmc_calib > $OUT/pmc_cf.log 2>&1 || { tail -30 $OUT/pmc_cf.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/calib_write -o run -- tools/pmc_calib > $OUT/pmc_cw.log 2>&1 || { tail -30 $OUT/pmc_cw.log; exit 1; }
python tools/collect_pmc.py $OUT/pmc --out $OUT/pmc_traffic.json --command "python3 $BENCH" > $OUT/collect.log 2>&1 || { cat $OUT/collect.log; exit 1; }
cat $OUT/pmc_traffic.json
# bench again, now reporting roofline.traffic from this box's counters
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python bench.py > $OUT/bench2.json 2> $OUT/bench2.err || { cat $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json
find $OUT/prof -name '*kernel_stats.csv' | head -5
