set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh lookback c2 "KCEP_STENCIL_ORDER=gather" "KCEP_STENCIL_ORDER=lookback" 3 --carry-batches 10 --processor-batch , || exit 1
bash tools/ab_env.sh lookback5 c5 "KCEP_STENCIL_ORDER=gather" "KCEP_STENCIL_ORDER=lookback" 2 --carry-batches 10 --processor-batch , || exit 1
echo done
