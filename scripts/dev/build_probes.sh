#!/bin/bash
# Build the cost-probe library (csrc/probes) in-tree: tensorflow_examples_amd/_lib/libtfx_probe.so.
set -e
cd "$(dirname "$0")/../.."
O=build/probes; mkdir -p $O
objs=""
for f in csrc/probes/*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Icsrc/include -Wno-unused-result \
    -c $f -o $O/$b.o &
  objs="$objs $O/$b.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tensorflow_examples_amd/_lib/libtfx_probe.so $objs
echo built
