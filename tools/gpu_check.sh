#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log || exit 1
timeout -k 10 300 python -u bench.py 2>&1 | tee gpurun_out/bench.log || exit 1
