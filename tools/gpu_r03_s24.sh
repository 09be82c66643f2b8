set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_carry_gpu.py -k "stencil" > gpurun_out/r03_s24_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s24_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s24_pytest.log
bash tools/ab_env.sh carrynoclaim c2 "KCEP_X=1" "KCEP_LIB=$PWD/build_variants/cw5/libkcep.so" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh carryvisit2 c2 "KCEP_X=1" "KCEP_CARRY_DBG=8" 1 --processor-batch , --carry-batches 10 || exit 1
echo done
