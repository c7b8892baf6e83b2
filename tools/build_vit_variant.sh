#!/bin/bash
# Diagnostic: link a variant library build/var/vit_<name>.so with lt_vit.hip
# built under extra flags (e.g. -DLT_VIT_WEARLY=0), the other objects from
# build/obj. Usage: tools/build_vit_variant.sh <name> [hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I last_torch_amd/csrc -I include "$@" \
  -c -o build/var/vit_$name.o last_torch_amd/csrc/lt_vit.hip
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build/var/vit_$name.so build/obj/lt_lattice.o \
  build/obj/lt_pipe.o build/obj/lt_chunk.o build/obj/lt_table.o build/obj/lt_producer.o \
  build/var/vit_$name.o build/obj/lt_tri.o build/obj/lt_joint.o build/obj/lt_inst_*.o
echo build/var/vit_$name.so
