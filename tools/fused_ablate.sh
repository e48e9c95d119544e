#!/bin/bash
# Profiling aid: builds libtrpo_engine variants with parts of the fused FVP (fused.hip) removed
# (FUSED_ABL bits, see fused.hip) next to the shipped library.  Results are wrong by design; only
# the fused kernel's time is of interest.  usage: bash tools/fused_ablate.sh <bits>...
set -e
cd "$(dirname "$0")/../trpo_amd/csrc"
for b in "$@"; do
  mkdir -p ../../build/fabl$b
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DFUSED_ABL=$b -x hip -c fused.hip -o ../../build/fabl$b/fused.o
  objs=$(ls ../../build/csrc/*.o | grep -v fused.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $objs ../../build/fabl$b/fused.o -shared -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib -o ../libtrpo_engine_fabl$b.so
done
