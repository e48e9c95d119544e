#!/bin/bash
# A/B and ablation builds: libtrpo_engine with one source file recompiled under extra -D flags (or from an
# alternative source file), next to the shipped library in trpo_amd/abl/ (git-ignored, travels to the GPU box).
#   bash tools/variant.sh <name> <file.hip> [-DFLAG=V ...]   ->  trpo_amd/abl/libtrpo_engine_<name>.so
# Use it with TRPO_ENGINE_LIB=trpo_amd/abl/libtrpo_engine_<name>.so (tools/gpu.sh ab).
set -e -o pipefail
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../trpo_amd/csrc"
make -s >/dev/null
mkdir -p ../../build/var_$NAME ../abl
base=$(basename $SRC)
obj=../../build/var_$NAME/$base.o
rm -f $obj   # a failed compile must not leave an older object to be linked
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. "$@" -x hip -c $SRC \
  -o $obj > ../../build/var_$NAME/$base.log 2>&1 || { cat ../../build/var_$NAME/$base.log; exit 1; }
grep -E "error|spill" ../../build/var_$NAME/$base.log || true
test -s $obj
objs=$(ls ../../build/csrc/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 $objs ../../build/var_$NAME/$base.o -shared -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o ../abl/libtrpo_engine_$NAME.so
echo "built trpo_amd/abl/libtrpo_engine_$NAME.so"
