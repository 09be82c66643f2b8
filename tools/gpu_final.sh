#!/bin/bash
# End-of-round check of the final build: full GPU suite, smoke, then the default bench line per config.
# Usage: tools/gpu_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/final/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/final/pytest_$TAG.log
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/final/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/final/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/final/smoke_$TAG.log
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/final/bench_${c}_$TAG.log 2>&1 || { tail -20 gpurun_out/final/bench_${c}_$TAG.log; exit 1; }
  tail -1 gpurun_out/final/bench_${c}_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), d["checksum"], d["roofline"]["frac"])' $c
done
