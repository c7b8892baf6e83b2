#!/bin/bash
# Diagnostic: link build/var/<name>.so from the product objects with one
# translation unit recompiled (extra hipcc flags, e.g. -DLT_VIT_NW=4).
#   tools/build_var.sh <name> <unit: lt_vit|lt_tri|...> [hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; unit=$2; shift 2
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c -o build/var/$name.o last_torch_amd/csrc/$unit.hip
objs=""
for o in build/obj/*.o; do
  [ "$(basename $o .o)" = "$unit" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build/var/$name.so $objs build/var/$name.o
echo build/var/$name.so
