set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s22_c2carry -o trace -- python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-input --processor-batch , --carry-batches 10 > gpurun_out/r03_s22.log 2>&1 || exit 1
echo done
