#!/bin/bash
# Build an A/B variant of libgnnea.so with one source recompiled under extra flags:
#   bash tools/dbg/build_variant.sh <name> <source.hip> <flags...>   -> gnn-mtl_amd/gnnea/libgnnea_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; src=$2; shift 2
C=$ROOT/gnn-mtl_amd/csrc; OBJ=$ROOT/build/obj; V=$ROOT/build/var_$name
mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics -I$ROOT/include "$@" -c $C/$src -o $V/${src%.hip}.o
objs=""
for o in $OBJ/*.o; do b=$(basename $o); if [ "$b" = "${src%.hip}.o" ]; then objs="$objs $V/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/gnn-mtl_amd/gnnea/libgnnea_$name.so $objs
echo built libgnnea_$name.so
