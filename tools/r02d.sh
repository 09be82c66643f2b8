set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_general_gpu.py tests/test_carry_gpu.py tests/test_processor_gpu.py tests/test_streams_gpu.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_r02d.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r02d.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_r02d.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_r02d.log 2>&1 || { tail -20 gpurun_out/bench_c4_r02d.log; exit 1; }
tail -1 gpurun_out/bench_c4_r02d.log | cut -c1-700
timeout -k 10 200 python -u tools/c4_profile.py > gpurun_out/c4_profile_r02d.log 2>&1 && head -12 gpurun_out/c4_profile_r02d.log
timeout -k 10 200 python -u tools/c4_single.py --top1 > gpurun_out/c4_single_r02d.log 2>&1 && cat gpurun_out/c4_single_r02d.log
