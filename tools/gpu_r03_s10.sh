set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s10_c4g -o trace -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-input --processor-batch , > gpurun_out/r03_s10_c4g.log 2>&1 || exit 1
bash tools/ab_env.sh c4gruns c4 "KCEP_GROUP_RUNS=16" "KCEP_GROUP_RUNS=64" 1 --processor-batch , || exit 1
bash tools/ab_env.sh c4gocc c4 "KCEP_NFA_WAVE_OCC=2" "KCEP_NFA_WAVE_OCC=4" 1 --processor-batch , || exit 1
timeout -k 10 400 python -u -m pytest tests/test_stencil_gpu.py tests/test_chain_gpu.py tests/test_carry_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_s10_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s10_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh fin c2 "KCEP_STENCIL_SCAN_GATHER=1" "KCEP_X=1" 3 --processor-batch , --carry-batches 10 || exit 1
echo done
