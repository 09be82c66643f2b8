set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_general_gpu.py tests/test_carry_gpu.py tests/test_seqagg_gpu.py tests/test_processor_gpu.py tests/test_runs_gpu.py tests/test_baseline_sizes_gpu.py tests/test_jni_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r03_s9_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03_s9_pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh c4grp c4 "KCEP_NFA_GROUPED=0" "KCEP_NFA_GROUPED=1" 2 --processor-batch , || exit 1
bash tools/ab_env.sh c4garena c4 "KCEP_GROUP_ARENA=512" "KCEP_GROUP_ARENA=2048" 1 --processor-batch , || exit 1
bash tools/ab_env.sh c3chunk c3 "KCEP_LIB=build_variants/base/libkcep.so" "KCEP_X=1" 1 --processor-batch , --carry-batches 10 || exit 1
echo done
