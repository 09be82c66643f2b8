#!/bin/bash
# PC sampling of one bench config's kernels (rocprofv3, stochastic where the device offers it).
# Usage: tools/pcsamp.sh TAG CONFIG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
TAG=${1:-pcs}; C=${2:-c4}
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list_avail.txt 2>&1 || true
grep -i -A12 "pc.sampl\|PC_SAMPL" gpurun_out/pcs/list_avail.txt | head -60
METHOD=${PCS_METHOD:-stochastic}; UNIT=${PCS_UNIT:-cycles}; IV=${PCS_INTERVAL:-1048576}
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
  --pc-sampling-interval $IV --output-format csv -d gpurun_out/pcs/$TAG -o pcs -- \
  python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , \
  > gpurun_out/pcs/${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/pcs/${TAG}.log
find gpurun_out/pcs/$TAG -type f | head
exit $rc
