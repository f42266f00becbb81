#!/bin/bash
# Build an A/B variant of libtcx.so: one source recompiled with extra -D flags, linked with the
# product objects into abtmp/libtcx_<name>.so (the product library is untouched).
# usage: tools/build_variant.sh <name> <source.hip> <flags...>
set -e
cd "$(dirname "$0")/../vae-diffusion-toy-crystals_amd/csrc"
name=$1; src=$2; shift 2
mkdir -p ../../abtmp build_var
CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $CXXFLAGS "$@" -c $src -o build_var/${name}_${src}.o
objs=$(ls build/*.o | grep -v "build/${src}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../abtmp/libtcx_${name}.so $objs build_var/${name}_${src}.o
echo "built abtmp/libtcx_${name}.so"
