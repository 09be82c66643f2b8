set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_stencil_gpu.py tests/test_baseline_sizes_gpu.py tests/test_streams_gpu.py tests/test_processor_gpu.py tests/test_shard_gpu.py tests/test_general_gpu.py -k "not golden and not random_general" -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_s17_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s17_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh compact c2 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 3 --processor-batch , --carry-batches 1 || exit 1
echo done
