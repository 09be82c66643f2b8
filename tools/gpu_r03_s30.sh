set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_carry_gpu.py -k stencil > gpurun_out/r03_s30_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s30_pytest.log; exit 1; }
KCEP_LIB=$PWD/build_variants/cw6/libkcep.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_carry_gpu.py -k stencil > gpurun_out/r03_s30b_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s30b_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s30_pytest.log gpurun_out/r03_s30b_pytest.log
B=KCEP_LIB=$PWD/build_variants
bash tools/ab_env.sh carrycall c2 "$B/inl/libkcep.so" "KCEP_X=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh carrycw c2 "$B/cw6/libkcep.so" "$B/cw5/libkcep.so" 2 --processor-batch , --carry-batches 10 || exit 1
echo done
