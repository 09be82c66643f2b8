#!/bin/bash
# GPU session: parity tests, then bench.py on every BASELINE config, then a
# kernel-trace of the general-path configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${c}_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_$TAG.log
done
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/${TAG}_$c -o trace -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${c}_$TAG.log 2>&1 || exit 1
done
echo done
