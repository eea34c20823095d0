#!/bin/bash
# Round-5 profile: a C4-only rocprofv3 kernel trace + stats ($TAG), then two
# SQ counter passes over the kernels in $RX (wave-cycle split, LDS, VALU).
# Every pass its own run and time limit; stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r05p}
mkdir -p $OUT
step() { echo "== $1 $(date +%T)"; }
C4ONLY="bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-phases --no-configs --no-secondary --no-c5 --no-streaming"
RX=${RX:-k_cmd_search|k_code_scatter|k_graph_tile}
rm -rf $OUT/prof_$TAG $OUT/pmcA_$TAG $OUT/pmcB_$TAG
step stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $C4ONLY > $OUT/prof_$TAG.log 2>&1 || { tail -30 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name '*kernel_trace.csv' -delete
tail -1 $OUT/prof_$TAG.log | cut -c1-300
if [ -n "$PMC" ]; then
  step pmcA
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/pmcA_$TAG -o run -- python3 $C4ONLY > $OUT/pmcA_$TAG.log 2>&1 || { tail -30 $OUT/pmcA_$TAG.log; exit 1; }
  step pmcB
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcB_$TAG -o run -- python3 $C4ONLY > $OUT/pmcB_$TAG.log 2>&1 || { tail -30 $OUT/pmcB_$TAG.log; exit 1; }
fi
step done
