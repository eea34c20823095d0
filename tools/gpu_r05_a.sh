#!/bin/bash
# Round-5 probe A: the key-order -> command-order transition microbenchmark
# (tools/scatter_bench) and two PMC passes over the C4 tile / search / union
# kernels (LDS conflicts, LDS issue stalls, wave-cycle split).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r05a}
mkdir -p $OUT
step() { echo "== $1 $(date +%T)"; }
C4ONLY="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-phases --no-configs --no-secondary --no-c5 --no-streaming"
RX='k_graph_tile|k_cmd_search|k_cmd_engine'
step scatter
timeout -k 10 120 tools/scatter_bench > $OUT/scatter_$TAG.jsonl 2>&1 || { tail -20 $OUT/scatter_$TAG.jsonl; exit 1; }
step pmcA
timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/pmcA_$TAG -o run -- python3 $C4ONLY > $OUT/pmcA_$TAG.log 2>&1 || { tail -30 $OUT/pmcA_$TAG.log; exit 1; }
step pmcB
timeout -k 10 240 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcB_$TAG -o run -- python3 $C4ONLY > $OUT/pmcB_$TAG.log 2>&1 || { tail -30 $OUT/pmcB_$TAG.log; exit 1; }
step done
