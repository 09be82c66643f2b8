#!/bin/bash
# GPU session: parity tests, bench, rocprofv3 kernel trace + separate PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || [ "$KEEP_GOING" = 1 -a $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u bench.py 2>&1 | tee gpurun_out/bench_$TAG.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/$TAG -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_trace_$TAG.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof/$TAG -o pmc_fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_fetch_$TAG.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof/$TAG -o pmc_write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_write_$TAG.log 2>&1 || exit 1
echo done
