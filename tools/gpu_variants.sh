#!/bin/bash
# Variant timings of the C2 stencil kernel (build_variants/*), then the chain
# parity tests on the default build.  Usage: tools/gpu_variants.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-var}
timeout -k 10 400 python -u tools/stencil_variants.py > gpurun_out/variants_$TAG.log 2>&1 || { tail -20 gpurun_out/variants_$TAG.log; exit 1; }
cat gpurun_out/variants_$TAG.log
echo done
