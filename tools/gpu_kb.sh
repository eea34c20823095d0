#!/bin/bash
# Single-view bucket path session: parity tests of the KeyDeps/engine paths,
# the C2 bench, and the kbbench phase breakdown (built on the box).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_keydeps_gpu.py tests/test_engine_gpu.py} -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/kbt.log 2>&1 || { tail -40 $OUT/kbt.log; exit 1; }
tail -2 $OUT/kbt.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.3g' % d['value'], 'ms', d['ms_per_step'], 'roofline', d['roofline'])"
if [ -n "$KB" ]; then
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ifantoch_amd/csrc tools/kbbench.cpp -o /tmp/kbbench -Lfantoch_amd -lfantoch_hip -Wl,-rpath,$PWD/fantoch_amd && KB_BINS=/tmp/kbbench timeout -k 10 200 bash tools/kbbench.sh > $OUT/kb.log 2>&1 || { tail -20 $OUT/kb.log; exit 1; }
  head -12 $OUT/kb.log
fi
