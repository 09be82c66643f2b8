set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_stencil_gpu.py tests/test_chain_gpu.py tests/test_carry_gpu.py tests/test_baseline_sizes_gpu.py tests/test_jni_gpu.py tests/test_processor_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_s16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s16_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh kdirect5 c5 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh kdirect2 c2 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 2 --processor-batch , --carry-batches 10 || exit 1
echo done
