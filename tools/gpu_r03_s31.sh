set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KCEP_GATHER_THREADS=64 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_chain_gpu.py > gpurun_out/r03_s31_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s31_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s31_pytest.log
bash tools/ab_env.sh gather64 c2 "KCEP_X=1" "KCEP_GATHER_THREADS=64" 3 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh gather128 c2 "KCEP_X=1" "KCEP_GATHER_THREADS=128" 2 --processor-batch , --carry-batches 10 || exit 1
echo done
