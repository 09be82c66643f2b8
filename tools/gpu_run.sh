#!/bin/bash
# One GPU session: the -m gpu parity tests (optionally a subset), then bench.py on
# the given configs.  Usage: tools/gpu_run.sh TAG "test-selection" "c2 c5"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
SEL=${2:-tests}
CFGS=${3:-c2}
if [ "$SEL" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
fi
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${c}_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_$TAG.log
done
echo done
