set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_r02c.log
[ $rc -eq 0 ] || exit 1
for w in 1 0; do
  KCEP_NFA_WAVE=$w timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_wave$w.log 2>&1 || { tail -20 gpurun_out/bench_c4_wave$w.log; exit 1; }
  tail -1 gpurun_out/bench_c4_wave$w.log | cut -c1-900
done
