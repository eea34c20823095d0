#!/bin/bash
# Round-5 profiles: a C4-only rocprofv3 kernel trace + stats, then separate
# FETCH_SIZE / WRITE_SIZE passes over the C4-only bench and over the C5 probe
# (every pass its own run, its own time limit), with the calibration kernels;
# summaries collected into gpurun_out/ (then copied to profiles/).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r05}
mkdir -p $OUT
C4ONLY="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-phases --no-configs --no-secondary --no-c5 --no-streaming"
C5="tools/c5_probe.py --steps 2"
step() { echo "== $1 $(date +%T)"; }
rm -rf $OUT/prof_$TAG $OUT/pmc_$TAG $OUT/pmc5_$TAG
step stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $C4ONLY > $OUT/prof_$TAG.log 2>&1 || { tail -30 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name '*kernel_trace.csv' -delete
step stats_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5_$TAG -o run -- python3 $C5 > $OUT/prof5_$TAG.log 2>&1 || { tail -30 $OUT/prof5_$TAG.log; exit 1; }
find $OUT/prof5_$TAG -name '*kernel_trace.csv' -delete
step pmc
for ctr in FETCH_SIZE WRITE_SIZE; do
  sub=$([ $ctr = FETCH_SIZE ] && echo fetch || echo write)
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$TAG/$sub -o run -- python3 $C4ONLY > $OUT/pmc_${sub}_$TAG.log 2>&1 || { tail -30 $OUT/pmc_${sub}_$TAG.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc5_$TAG/$sub -o run -- python3 $C5 > $OUT/pmc5_${sub}_$TAG.log 2>&1 || { tail -30 $OUT/pmc5_${sub}_$TAG.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$TAG/calib_$sub -o run -- tools/pmc_calib > $OUT/pmc_c${sub}_$TAG.log 2>&1 || { tail -30 $OUT/pmc_c${sub}_$TAG.log; exit 1; }
done
cp -r $OUT/pmc_$TAG/calib_fetch $OUT/pmc5_$TAG/ && cp -r $OUT/pmc_$TAG/calib_write $OUT/pmc5_$TAG/
python tools/collect_pmc.py $OUT/pmc_$TAG --out $OUT/pmc_traffic_$TAG.json --command "python3 $C4ONLY" > $OUT/collect_$TAG.log 2>&1 || { cat $OUT/collect_$TAG.log; exit 1; }
python tools/collect_pmc.py $OUT/pmc5_$TAG --out $OUT/pmc_traffic_c5_$TAG.json --command "python3 $C5" > $OUT/collect5_$TAG.log 2>&1 || { cat $OUT/collect5_$TAG.log; exit 1; }
find $OUT/pmc_$TAG $OUT/pmc5_$TAG -name '*.csv' -size +20M -delete
step done
