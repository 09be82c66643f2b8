set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/c4_profile.py > gpurun_out/c4_profile_r02e.log 2>&1 && head -3 gpurun_out/c4_profile_r02e.log && grep "phase" gpurun_out/c4_profile_r02e.log
for o in 2 3 4 5 6 8; do
  KCEP_NFA_WAVE_OCC=$o timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_occ$o.log 2>&1 || { tail -5 gpurun_out/bench_c4_occ$o.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_c4_occ$o.log').read().strip().splitlines()[-1]); print('occ $o', d['ms_per_step'], d['checksum'])"
done
