set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_t5.log 2>&1
rc=$?; tail -5 gpurun_out/r03_t5.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh c4r02 c4 "KCEP_LIB=build_variants/r02/libkcep.so" "KCEP_X=1" 2 || exit 1
bash tools/ab_env.sh c4mid c4 "KCEP_LIB=build_variants/mid/libkcep.so" "KCEP_X=1" 1 || exit 1
bash tools/ab_env.sh c4priv c4 "KCEP_WAVE_PRIV=0" "KCEP_WAVE_PRIV=16" 2 || exit 1
bash tools/ab_env.sh c3gen c3 "KCEP_X=1" "KCEP_X=1" 1 --force-path general --nfa-kernel wave || exit 1
bash tools/ab_env.sh c3genl c3 "KCEP_X=1" "KCEP_X=1" 1 --force-path general --nfa-kernel lane || exit 1
echo done
