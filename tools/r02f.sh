set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_carry_gpu.py tests/test_processor_gpu.py tests/test_stencil_gpu.py tests/test_chain_gpu.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_r02f.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r02f.log
[ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" gpurun_out/pytest_r02f.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-host-input > gpurun_out/bench_c2_r02f.log 2>&1 || { tail -20 gpurun_out/bench_c2_r02f.log; exit 1; }
tail -1 gpurun_out/bench_c2_r02f.log | cut -c1-400
