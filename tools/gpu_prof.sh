#!/bin/bash
# rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE PMC passes of
# bench.py for each config.  Usage: tools/gpu_prof.sh TAG "c2 c5 c3"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
for c in ${2:-c2}; do
  D=gpurun_out/prof/${TAG}_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o trace -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/prof_trace_${TAG}_$c.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D -o pmc_fetch -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/prof_fetch_${TAG}_$c.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D -o pmc_write -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/prof_write_${TAG}_$c.log 2>&1 || exit 1
  echo "profiled $c"
done
echo done
