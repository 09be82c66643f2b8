#!/bin/bash
# A/B of an environment switch on one build: tools/ab_env.sh "VAR=value" [config] (alternating runs on one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
C=${2:-c4}
for i in 1 2 3; do
  env $1 timeout -k 10 200 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/old_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/new_$i.log 2>&1 || exit 1
  echo "round $i done"
done
