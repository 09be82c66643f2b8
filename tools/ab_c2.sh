#!/bin/bash
# A/B of two libkcep.so builds on the C2 bench (alternating runs on one box).
# Usage: tools/ab_c2.sh OLD_SO [config]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
C=${2:-c2}
for i in 1 2 3; do
  KCEP_LIB=$1 timeout -k 10 200 python -u bench.py --config $C --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/old_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config $C --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/new_$i.log 2>&1 || exit 1
  echo "round $i done"
done
