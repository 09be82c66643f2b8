set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_runs_gpu.py tests/test_carry_gpu.py tests/test_baseline_sizes_gpu.py tests/test_seqagg_gpu.py tests/test_processor_gpu.py > gpurun_out/r03_s29_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s29_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s29_pytest.log
bash tools/ab_env.sh runsorder c3 "KCEP_RUNS_RADIX=1" "KCEP_X=1" 3 || exit 1
echo done
