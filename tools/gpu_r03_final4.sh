set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_final4_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_final4_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final4_smoke.log 2>&1 || { tail -5 gpurun_out/r03_final4_smoke.log; exit 1; }
tail -1 gpurun_out/r03_final4_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03_final4_bench_c2.log 2>&1 || { tail -5 gpurun_out/r03_final4_bench_c2.log; exit 1; }
tail -1 gpurun_out/r03_final4_bench_c2.log | cut -c1-300
for c in c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/r03_final4_bench_$c.log 2>&1 || { tail -5 gpurun_out/r03_final4_bench_$c.log; exit 1; }
  tail -1 gpurun_out/r03_final4_bench_$c.log | cut -c1-250
done
echo done
