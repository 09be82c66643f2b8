set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_env.sh early c2 "KCEP_LIB=build_variants/late/libkcep.so" "KCEP_X=1" 3 --carry-batches 1 --processor-batch , || exit 1
bash tools/ab_env.sh w7 c2 "KCEP_LIB=build_variants/w7/libkcep.so" "KCEP_STENCIL_KEYED=1" 2 --carry-batches 1 --processor-batch , || exit 1
echo done
