set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_general_gpu.py tests/test_seqagg_gpu.py tests/test_carry_gpu.py -k "capacity or stencil or chain" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_t2.log 2>&1
rc=$?; tail -5 gpurun_out/r03_t2.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh stwave c2 "KCEP_STENCIL=wg" "KCEP_STENCIL=wave" 3 --carry-batches 1 || exit 1
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_c3.log 2>&1 || { tail -5 gpurun_out/r03_c3.log; exit 1; }
tail -1 gpurun_out/r03_c3.log | cut -c1-700
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_c2.log 2>&1 || { tail -5 gpurun_out/r03_c2.log; exit 1; }
tail -1 gpurun_out/r03_c2.log
