set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh ntstore c2 "KCEP_X=1" "KCEP_LIB=build_variants/ntstore/libkcep.so" 3 --processor-batch , --carry-batches 1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_s14_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s14_pytest.log; [ $rc -eq 0 ] || exit 1
echo done
