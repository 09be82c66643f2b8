set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_stencil_gpu.py tests/test_baseline_sizes_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_s12_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s12_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh defer c2 "KCEP_LIB=build_variants/immediate/libkcep.so" "KCEP_X=1" 3 --processor-batch , --carry-batches 1 || exit 1
echo done
