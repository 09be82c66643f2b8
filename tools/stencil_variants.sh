#!/bin/bash
# Build stencil-kernel variants (compile-time knobs on csrc/stencil.hip only) as
# separate libkcep.so files under build_variants/<name>/, linked with the other
# objects of the current in-tree build, for tools/stencil_variants.py.
set -e
cd "$(dirname "$0")/.."
make -s -C kafkastreams-cep_amd -j8 >/dev/null
B=kafkastreams-cep_amd/build
F="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result"
rm -rf build_variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_variants/$name
  O=build_variants/$name/stencil.o
  /opt/rocm/bin/hipcc $F $flags -x hip -c kafkastreams-cep_amd/csrc/stencil.hip -o $O
  /opt/rocm/bin/hipcc $F -shared -o build_variants/$name/libkcep.so $B/compile.cpp.o $B/abi.cpp.o $B/jit.cpp.o \
    $B/nfa.hip.o $B/runs.hip.o $O -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
  rm $O
done
