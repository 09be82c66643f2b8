set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_carry_gpu.py tests/test_chain_gpu.py > gpurun_out/r03_s26_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s26_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s26_pytest.log
bash tools/ab_env.sh carryrep c2 "KCEP_X=1" "KCEP_CARRY_DBG=8" 2 --processor-batch , --carry-batches 10 || exit 1
echo done
