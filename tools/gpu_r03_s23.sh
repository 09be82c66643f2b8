set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh carryvisit c2 "KCEP_X=1" "KCEP_CARRY_DBG=8" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh ev10m c2 "KCEP_X=1" "KCEP_STENCIL_KEYED=1" 2 --processor-batch , --carry-batches 1 --events 10000000 || exit 1
echo done
