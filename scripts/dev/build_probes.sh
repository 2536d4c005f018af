#!/bin/bash
# Build the cost-probe library (csrc/probes) in-tree: tensorflow_examples_amd/_lib/libtfx_probe.so.
set -e
cd "$(dirname "$0")/../.."
O=build/probes; mkdir -p $O
for v in atomic store; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Icsrc/include -Wno-unused-result \
    -c csrc/probes/igemm_splitk_probe_$v.hip -o $O/probe_$v.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tensorflow_examples_amd/_lib/libtfx_probe.so $O/probe_atomic.o $O/probe_store.o
echo built
