set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py tests/test_baseline_sizes_gpu.py tests/test_streams_gpu.py tests/test_processor_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_s4_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03_s4_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh plain c2 "KCEP_STENCIL_KEYED=1" "KCEP_STENCIL_KEYED=0" 3 --carry-batches 1 --processor-batch , || exit 1
echo done
