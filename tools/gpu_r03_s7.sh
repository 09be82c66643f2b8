set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_runs_gpu.py tests/test_carry_gpu.py -k "runs" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_s7_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s7_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh c3pf c3 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 2 --processor-batch , --carry-batches 1 || exit 1
bash tools/ab_env.sh c4p0 c4 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 2 --processor-batch , || exit 1
bash tools/ab_env.sh c4ar c4 "KCEP_WAVE_ARENA=1536" "KCEP_WAVE_ARENA=3072" 1 --processor-batch , || exit 1

timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s8_c2carry -o trace -- python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 10 --no-host-input --processor-batch , > gpurun_out/r03_s8_c2carry.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r03s8_c3carry -o trace -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --carry-batches 10 --no-host-input --processor-batch , > gpurun_out/r03_s8_c3carry.log 2>&1 || exit 1
echo done
