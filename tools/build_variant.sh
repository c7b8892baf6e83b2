#!/bin/bash
# Diagnostic: link a variant library build/var/<name>.so from a modified copy
# of lt_chunk.hip (the other objects from build/obj). Usage:
#   tools/build_variant.sh <name> <path-to-lt_chunk-variant.hip> [hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I last_torch_amd/csrc -I include "$@" -c -o build/var/$name.o "$src"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build/var/$name.so build/obj/lt_lattice.o build/obj/lt_pipe.o build/var/$name.o build/obj/lt_table.o build/obj/lt_producer.o build/obj/lt_joint.o build/obj/lt_vit.o build/obj/lt_tri.o build/obj/lt_inst_*.o
echo build/var/$name.so
