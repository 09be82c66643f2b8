set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_stencil_gpu.py tests/test_chain_gpu.py tests/test_carry_gpu.py tests/test_runs_gpu.py tests/test_shard_gpu.py tests/test_processor_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_s11_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s11_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/bw_probe > gpurun_out/r03_s11_bw_probe.log 2>&1 || exit 1
cat gpurun_out/r03_s11_bw_probe.log
for v in nohit nowrite both; do
  bash tools/ab_env.sh probe_$v c2 "KCEP_X=1" "KCEP_LIB=build_variants/$v/libkcep.so" 2 --processor-batch , --carry-batches 1 || exit 1
done
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --processor-batch , > gpurun_out/r03_s11_c3.log 2>&1 || exit 1
tail -1 gpurun_out/r03_s11_c3.log | cut -c1-200
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --processor-batch , > gpurun_out/r03_s11_c2.log 2>&1 || exit 1
tail -1 gpurun_out/r03_s11_c2.log | cut -c1-200
echo done
