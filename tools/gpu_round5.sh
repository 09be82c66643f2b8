#!/bin/bash
# Round-5 check: full GPU suite, then C3 bench (runs_emit) and C4 bench; one line each.
# Usage: tools/gpu_round5.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for c in ${CONFIGS:-c3 c4}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${c}_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); cs=d.get("carry_stream") or {}; print(sys.argv[1], round(d["ms_per_step"],4), d["checksum"], d["first_kernel"], "carry", cs.get("ms_per_pass"), cs.get("vs_resident"), cs.get("parity"))' $c
done
