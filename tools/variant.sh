#!/bin/bash
# A/B and ablation builds: libtrpo_engine with one source file recompiled under extra -D flags (or from an
# alternative source file), next to the shipped library in trpo_amd/abl/ (git-ignored, travels to the GPU box).
#   bash tools/variant.sh <name> <file.hip> [-DFLAG=V ...]   ->  trpo_amd/abl/libtrpo_engine_<name>.so
# Use it with TRPO_ENGINE_LIB=trpo_amd/abl/libtrpo_engine_<name>.so (tools/gpu.sh ab).
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../trpo_amd/csrc"
make -s >/dev/null
mkdir -p ../../build/var_$NAME ../abl
base=$(basename $SRC)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. "$@" -x hip -c $SRC \
  -o ../../build/var_$NAME/$base.o 2>&1 | grep -E "error|spill" || true
objs=$(ls ../../build/csrc/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 $objs ../../build/var_$NAME/$base.o -shared -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o ../abl/libtrpo_engine_$NAME.so
echo "built trpo_amd/abl/libtrpo_engine_$NAME.so"
