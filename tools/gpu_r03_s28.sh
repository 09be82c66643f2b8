set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_carry_gpu.py -k "topic_and_wide or large_batches" > gpurun_out/r03_s28_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s28_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s28_pytest.log
bash tools/gpu_r03_final3_b.sh || exit 1
