set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_carry_gpu.py tests/test_stencil_gpu.py tests/test_processor_gpu.py tests/test_streams_gpu.py tests/test_jni_gpu.py tests/test_shard_gpu.py > gpurun_out/r03_s20_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s20_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s20_pytest.log
bash tools/ab_env.sh carryplain c2 "KCEP_STENCIL_KEYED=1" "KCEP_X=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh carryw5 c2 "KCEP_X=1" "KCEP_LIB=$PWD/build_variants/cw5/libkcep.so" 2 --processor-batch , --carry-batches 10 || exit 1
echo done
