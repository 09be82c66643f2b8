set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KCEP_STENCIL_FUSED_SCAN=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_carry_gpu.py tests/test_baseline_sizes_gpu.py tests/test_processor_gpu.py > gpurun_out/r03_s27_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s27_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s27_pytest.log
bash tools/ab_env.sh fusescan c2 "KCEP_X=1" "KCEP_STENCIL_FUSED_SCAN=1" 3 --processor-batch , --carry-batches 10 || exit 1
echo done
