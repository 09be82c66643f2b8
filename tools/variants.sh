#!/bin/bash
# Build libkcep.so variants that differ in compile-time knobs of ONE translation unit, linked with
# the other objects of the in-tree build, as build_variants/<name>/libkcep.so (A/B with KCEP_LIB=...).
# Usage: tools/variants.sh UNIT[,UNIT...] "name:flags" ...   e.g. tools/variants.sh stencil_k3 "late:-DST_PLAIN_EARLY=0"
set -e
cd "$(dirname "$0")/.."
make -s -C kafkastreams-cep_amd -j8 >/dev/null
B=kafkastreams-cep_amd/build
U=$1; shift
F="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_variants/$name
  objs=$(ls $B/*.o); O=""
  for u in ${U//,/ }; do
    /opt/rocm/bin/hipcc $F $flags -x hip -c kafkastreams-cep_amd/csrc/$u.hip -o build_variants/$name/$u.o
    objs=$(echo "$objs" | grep -v "/$u.hip.o$"); O="$O build_variants/$name/$u.o"
  done
  /opt/rocm/bin/hipcc $F -shared -o build_variants/$name/libkcep.so $objs $O -L/opt/rocm/lib -lhiprtc -ldl -Wl,-rpath,/opt/rocm/lib
  rm $O
done
