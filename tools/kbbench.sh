#!/bin/bash
# Diagnostic: C2 batch (Zipf 0.7 over 2^20 keys, 1M commands) through kbbench.
set -e
cd "$(dirname "$0")/.."
python - << 'PY'
import numpy as np
from fantoch_amd.workload import Workload
s = Workload.zipf(0.7, 1 << 20, k=1).generate(1_000_000)
s.keys[:, 0].astype(np.uint32).tofile("/tmp/kb_keys.u32")
s.dots.astype(np.uint64).tofile("/tmp/kb_dots.u64")
PY
for b in ${KB_BINS:-tools/kbbench}; do echo "== $b"; timeout -k 10 60 $b /tmp/kb_keys.u32 /tmp/kb_dots.u64 1000000 20 20; done
