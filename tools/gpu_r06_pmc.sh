#!/bin/bash
# Round-6 counters on the C4-only bench: separate FETCH_SIZE / WRITE_SIZE
# passes with the calibration kernels (tools/collect_pmc.py), then two SQ
# passes over the tile kernel, the search and the row placement.  Every pass
# its own run and time limit; stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r06m}
mkdir -p $OUT
C4ONLY="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-phases --no-configs --no-secondary --no-c5 --no-streaming"
RX=${RX:-k_cmd_search|k_row_place|k_graph_tile}
step() { echo "== $1 $(date +%T)"; }
rm -rf $OUT/pmc_$TAG $OUT/pmcA_$TAG $OUT/pmcB_$TAG
step pmc
for ctr in FETCH_SIZE WRITE_SIZE; do
  sub=$([ $ctr = FETCH_SIZE ] && echo fetch || echo write)
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$TAG/$sub -o run -- python3 $C4ONLY > $OUT/pmc_${sub}_$TAG.log 2>&1 || { tail -30 $OUT/pmc_${sub}_$TAG.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$TAG/calib_$sub -o run -- tools/pmc_calib > $OUT/pmc_c${sub}_$TAG.log 2>&1 || { tail -30 $OUT/pmc_c${sub}_$TAG.log; exit 1; }
done
python tools/collect_pmc.py $OUT/pmc_$TAG --out $OUT/pmc_traffic_$TAG.json --command "python3 $C4ONLY" > $OUT/collect_$TAG.log 2>&1 || { cat $OUT/collect_$TAG.log; exit 1; }
find $OUT/pmc_$TAG -name '*.csv' -size +20M -delete
step pmcA
timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/pmcA_$TAG -o run -- python3 $C4ONLY > $OUT/pmcA_$TAG.log 2>&1 || { tail -30 $OUT/pmcA_$TAG.log; exit 1; }
step pmcB
timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcB_$TAG -o run -- python3 $C4ONLY > $OUT/pmcB_$TAG.log 2>&1 || { tail -30 $OUT/pmcB_$TAG.log; exit 1; }
find $OUT/pmcA_$TAG $OUT/pmcB_$TAG -name '*.csv' -size +20M -delete
step done
