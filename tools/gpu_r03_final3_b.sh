set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof.sh r03final3 "c2 c5 c3 c4" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r03_final3b_bench_c2.log 2>&1 || { tail -5 gpurun_out/r03_final3b_bench_c2.log; exit 1; }
tail -1 gpurun_out/r03_final3b_bench_c2.log | cut -c1-300
echo done
