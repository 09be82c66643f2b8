set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_carry_gpu.py -k "stencil" > gpurun_out/r03_s25_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s25_pytest.log; exit 1; }
KCEP_STENCIL_SUB=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_carry_gpu.py -k "stencil" > gpurun_out/r03_s25b_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s25b_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s25_pytest.log gpurun_out/r03_s25b_pytest.log
bash tools/ab_env.sh carrysub c2 "KCEP_X=1" "KCEP_STENCIL_SUB=4" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh ev10msub c2 "KCEP_X=1" "KCEP_STENCIL_SUB=4" 1 --processor-batch , --carry-batches 1 --events 10000000 || exit 1
echo done
