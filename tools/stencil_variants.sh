#!/bin/bash
# Build stencil-kernel variants (compile-time knobs on csrc/stencil_k$K.hip, K = ${K:-3}: C2) as
# separate libkcep.so files under build_variants/<name>/, linked with the other objects of the
# current in-tree build, for tools/stencil_variants.py.  usage: stencil_variants.sh name:"-DX=1" ...
set -e
cd "$(dirname "$0")/.."
K=${K:-3}
make -s -C kafkastreams-cep_amd -j8 >/dev/null
B=kafkastreams-cep_amd/build
F="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off"
rm -rf build_variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_variants/$name
  O=build_variants/$name/stencil_k$K.o
  O2=build_variants/$name/stencil.o            # the slot consumers see the same knobs
  /opt/rocm/bin/hipcc $F $flags -I include -x hip -c kafkastreams-cep_amd/csrc/stencil_k$K.hip -o $O
  /opt/rocm/bin/hipcc $F $flags -I include -x hip -c kafkastreams-cep_amd/csrc/stencil.hip -o $O2
  objs=$(ls $B/*.o | grep -v "stencil_k$K.hip.o\|/stencil.hip.o")
  /opt/rocm/bin/hipcc $F -shared -o build_variants/$name/libkcep.so $objs $O $O2 -L/opt/rocm/lib -lhiprtc -ldl \
    -Wl,-rpath,/opt/rocm/lib
  rm $O $O2
done
