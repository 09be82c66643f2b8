set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_t4.log 2>&1
rc=$?; tail -15 gpurun_out/r03_t4.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh stwave c2 "KCEP_STENCIL=wg" "KCEP_STENCIL=wave" 3 --carry-batches 1 || exit 1
bash tools/ab_env.sh c4priv c4 "KCEP_WAVE_PRIV=0" "KCEP_WAVE_PRIV=16" 2 || exit 1
bash tools/ab_env.sh c3gen c3 "KCEP_NFA_WAVE_AGG=0" "KCEP_NFA_WAVE_AGG=1" 1 --force-path general || exit 1
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_c3.log 2>&1 || { tail -5 gpurun_out/r03_c3.log; exit 1; }
tail -1 gpurun_out/r03_c3.log | cut -c1-3000
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_c2.log 2>&1 || { tail -5 gpurun_out/r03_c2.log; exit 1; }
tail -1 gpurun_out/r03_c2.log
