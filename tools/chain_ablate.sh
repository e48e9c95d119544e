#!/bin/bash
# Profiling aid: builds libtrpo_engine variants with parts of the fused FVP chain removed
# (CHAIN_ABL bits, see chain.hip) next to the shipped library.  Results are wrong by design;
# only the chain kernel's time is of interest.  usage: bash tools/chain_ablate.sh <bits>...
set -e
cd "$(dirname "$0")/../trpo_amd/csrc"
for b in "$@"; do
  mkdir -p ../../build/abl$b
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DCHAIN_ABL=$b -x hip -c chain.hip -o ../../build/abl$b/chain.o
  objs=$(ls ../../build/csrc/*.o | grep -v chain.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $objs ../../build/abl$b/chain.o -shared -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib -o ../libtrpo_engine_abl$b.so
done
