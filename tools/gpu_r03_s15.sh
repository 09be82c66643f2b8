set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh direct c2 "KCEP_X=1" "KCEP_LIB=build_variants/direct/libkcep.so" 3 --processor-batch , --carry-batches 1 || exit 1
bash tools/ab_env.sh c4occ4 c4 "KCEP_X=1" "KCEP_NFA_WAVE_OCC=4 KCEP_WAVE_ARENA=1536" 2 --processor-batch , || exit 1
bash tools/ab_env.sh c4occ4b c4 "KCEP_NFA_WAVE_OCC=4" "KCEP_NFA_WAVE_OCC=5 KCEP_WAVE_ARENA=1024" 1 --processor-batch , || exit 1
echo done
