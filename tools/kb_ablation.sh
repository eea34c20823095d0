set -e
cd "$(dirname "$0")/.."
for v in base NOCLOCK; do
  F=""; [ $v != base ] && F="-DFH_ABL_$v"
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 $F -Iinclude -Ifantoch_amd/csrc tools/kbbench.cpp -o /tmp/kb_$v -Lfantoch_amd -lfantoch_hip -Wl,-rpath,$PWD/fantoch_amd &
done
wait
KB_BINS="/tmp/kb_base /tmp/kb_NOCLOCK" timeout -k 10 200 bash tools/kbbench.sh > gpurun_out/kbab.log 2>&1
grep -E "==|kb_partition: avg|partition phases" gpurun_out/kbab.log
