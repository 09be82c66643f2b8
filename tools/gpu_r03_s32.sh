set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_chain_gpu.py tests/test_carry_gpu.py > gpurun_out/r03_s32_pytest.log 2>&1 || { tail -40 gpurun_out/r03_s32_pytest.log; exit 1; }
tail -1 gpurun_out/r03_s32_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_s32_smoke.log 2>&1 || { tail -5 gpurun_out/r03_s32_smoke.log; exit 1; }
tail -1 gpurun_out/r03_s32_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03_s32_bench_c2.log 2>&1 || { tail -5 gpurun_out/r03_s32_bench_c2.log; exit 1; }
tail -1 gpurun_out/r03_s32_bench_c2.log | cut -c1-200
echo done
