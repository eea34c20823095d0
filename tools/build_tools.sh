#!/bin/bash
# Builds the standalone tool binaries against the in-tree library.
set -e
cd "$(dirname "$0")/.."
python -m fantoch_amd.build
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 tools/pmc_calib.hip -o tools/pmc_calib
/opt/rocm/bin/hipcc -O3 -std=c++17 -Iinclude tools/stream_bench.cpp -o tools/stream_bench -Lfantoch_amd -lfantoch_hip -Wl,-rpath,'$ORIGIN/../fantoch_amd'
