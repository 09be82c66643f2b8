set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh carrydbg1 c2 "KCEP_X=1" "KCEP_CARRY_DBG=1" 2 --processor-batch , --carry-batches 10 || exit 1
bash tools/ab_env.sh carrydbg7 c2 "KCEP_CARRY_DBG=2" "KCEP_CARRY_DBG=7" 1 --processor-batch , --carry-batches 10 || exit 1
echo done
