#!/bin/bash
# C4: parity tests of the general path, then alternating bench runs of env variants (A/B on one box).
# Usage: tools/gpu_c4ab.sh TAG "ENV1" "ENV2" ...   (ENV: space-free VAR=VALUE list joined by commas, or -)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
TAG=$1; shift
[ -n "$SKIP_TESTS" ] || { timeout -k 10 700 python -u -m pytest tests/test_general_gpu.py tests/test_seqagg_gpu.py tests/test_handoff_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log; }
for r in 1 2; do
  for v in "$@"; do
    envs=$(echo "$v" | tr ',' ' '); [ "$v" = "-" ] && envs=""
    env $envs timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --handoff-cap 0 > gpurun_out/ab/${TAG}_${r}_$(echo "$v" | tr -c "A-Za-z0-9\n" _).log 2>&1 || { tail -5 gpurun_out/ab/${TAG}_${r}_*.log; exit 1; }
    echo "[$v] run $r $(tail -1 gpurun_out/ab/${TAG}_${r}_$(echo "$v" | tr -c "A-Za-z0-9\n" _).log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["checksum"], round(d["first_kernel"]["ms"],3))')"
  done
done
