#!/bin/bash
# Round-3 GPU session: the GPU suite (with the C5 100M test), smoke, the full
# bench line, then C4-only profiles -- rocprofv3 kernel trace + stats and the
# FETCH_SIZE / WRITE_SIZE passes (each its own run) with the calibration
# kernels -- so per-launch figures are C4 figures.  Every GPU step has its
# own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r03}
C4ONLY="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-phases --no-configs --no-secondary --no-c5"
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --durations=20 --timeout 600 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -28 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { cat $OUT/smoke_$TAG.log; exit 1; }
  cat $OUT/smoke_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench
  timeout -k 10 600 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
if [ -z "$SKIP_PROF" ]; then
  rm -rf $OUT/prof_$TAG $OUT/pmc_$TAG
  step rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $C4ONLY > $OUT/prof_$TAG.log 2>&1 || { tail -30 $OUT/prof_$TAG.log; exit 1; }
  tail -1 $OUT/prof_$TAG.log
  python tools/attribute_copies.py "$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)" > $OUT/copybuffer_$TAG.json || exit 1
  find $OUT/prof_$TAG -name '*kernel_trace.csv' -delete
  step pmc
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/fetch -o run -- python3 $C4ONLY > $OUT/pmc_fetch_$TAG.log 2>&1 || { tail -30 $OUT/pmc_fetch_$TAG.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/write -o run -- python3 $C4ONLY > $OUT/pmc_write_$TAG.log 2>&1 || { tail -30 $OUT/pmc_write_$TAG.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/calib_fetch -o run -- tools/pmc_calib > $OUT/pmc_cf_$TAG.log 2>&1 || { tail -30 $OUT/pmc_cf_$TAG.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/calib_write -o run -- tools/pmc_calib > $OUT/pmc_cw_$TAG.log 2>&1 || { tail -30 $OUT/pmc_cw_$TAG.log; exit 1; }
  python tools/collect_pmc.py $OUT/pmc_$TAG --out $OUT/pmc_traffic_$TAG.json --command "python3 $C4ONLY" > $OUT/collect_$TAG.log 2>&1 || { cat $OUT/collect_$TAG.log; exit 1; }
  step done
fi
