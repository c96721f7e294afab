#!/bin/bash
# Experimental lstm_batch.hip variants (LB_DBG bits: 1 no output stores, 2 no input loads)
# linked with the working-tree objects as ab/libensvs_lbN.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p ab
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iensemble_svs_with_interactions_amd/csrc -Iinclude \
    -DLB_DBG=$n -c ensemble_svs_with_interactions_amd/csrc/lstm_batch.hip -o ab/lb_$n.o &
done
wait
for n in "$@"; do
  objs=$(ls build/*.o | grep -v lstm_batch.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/libensvs_lb$n.so $objs ab/lb_$n.o
done
