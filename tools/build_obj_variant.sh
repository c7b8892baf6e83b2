#!/bin/bash
# Diagnostic: link a variant library build/var/<obj>_<name>.so in which
# lt_<obj>.hip is built under extra flags (e.g. -DLT_PIPE_NAP=4) and every
# other object comes from build/obj. Usage:
#   tools/build_obj_variant.sh <obj> <name> [hipcc flags]
set -e
cd "$(dirname "$0")/.."
obj=$1; name=$2; shift 2
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I last_torch_amd/csrc -I include "$@" \
  -c -o build/var/${obj}_$name.o last_torch_amd/csrc/lt_$obj.hip
objs=""
for o in build/obj/lt_*.o; do
  [ "$o" = build/obj/lt_$obj.o ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build/var/${obj}_$name.so $objs build/var/${obj}_$name.o
echo build/var/${obj}_$name.so
