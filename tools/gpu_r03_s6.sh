set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh c4priv c4 "KCEP_WAVE_PRIV=0" "KCEP_WAVE_PRIV=16" 2 --processor-batch , || exit 1
bash tools/ab_env.sh c4arena c4 "KCEP_WAVE_ARENA=1536" "KCEP_WAVE_ARENA=2048" 1 --processor-batch , || exit 1
bash tools/gpu_prof.sh r03s6 "c3 c4" || exit 1
echo done
