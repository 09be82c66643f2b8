set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s8_c2carry -o trace -- python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 10 --no-host-input --processor-batch , > gpurun_out/r03_s8_c2carry.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s8_c3carry -o trace -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 10 --no-host-input --processor-batch , > gpurun_out/r03_s8_c3carry.log 2>&1 || exit 1
echo done
