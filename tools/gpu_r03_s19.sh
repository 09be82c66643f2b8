set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_chain_gpu.py tests/test_carry_gpu.py tests/test_baseline_sizes_gpu.py tests/test_processor_gpu.py > gpurun_out/r03_s19_pytest.log 2>&1 || { tail -30 gpurun_out/r03_s19_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s19_pytest.log
B=KCEP_LIB=$PWD/build_variants/base/libkcep.so
bash tools/ab_env.sh c5compact c5 "$B" "KCEP_X=1" 3 || exit 1
bash tools/ab_env.sh c2carrycompact c2 "$B" "KCEP_X=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh c2compact c2 "$B" "KCEP_X=1" 2 || exit 1
bash tools/ab_env.sh carrydbg1 c2 "KCEP_X=1" "KCEP_CARRY_DBG=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh carrydbg7 c2 "KCEP_CARRY_DBG=2" "KCEP_CARRY_DBG=7" 1 --processor-batch , --carry-batches 10 || exit 1
echo done
