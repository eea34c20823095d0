#!/bin/bash
# HBM traffic of the C4 headline kernels: separate FETCH_SIZE / WRITE_SIZE
# rocprofv3 passes over bench.py and over tools/pmc_calib (per-width
# calibration on the same box), then tools/collect_pmc.py ->
# profiles/pmc_traffic.json (bench.py's roofline.traffic).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=gpurun_out/pmc
rm -rf $R; mkdir -p $R
if [ -n "$CFG" ]; then   # a tools/bench_configs.py configuration (e.g. CFG=c5)
  PROG="tools/bench_configs.py"; ARGS="--only $CFG --no-cpu --steps 1 --warmup 0"
else
  PROG="bench.py"; ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-phases"
fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 $PROG $ARGS > $R/fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $R/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 $PROG $ARGS > $R/write.log 2>&1 || { echo "write pass failed"; tail -5 $R/write.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/calib_fetch -o run -- tools/pmc_calib > $R/cf.log 2>&1 || { echo "calib fetch failed"; tail -5 $R/cf.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/calib_write -o run -- tools/pmc_calib > $R/cw.log 2>&1 || { echo "calib write failed"; tail -5 $R/cw.log; exit 1; }
OUTF=profiles/pmc_traffic${CFG:+_$CFG}.json
python3 tools/collect_pmc.py $R --out $OUTF --command "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- python3 $PROG $ARGS; tools/pmc_calib" > $R/collect.log 2>&1 || { cat $R/collect.log; exit 1; }
cp $OUTF gpurun_out/$(basename $OUTF)
cat gpurun_out/$(basename $OUTF)
