set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg_carry.py 2 1 && KCEP_STENCIL_KEYED=1 timeout -k 10 120 python -u tools/dbg_carry.py 2 1 && timeout -k 10 120 python -u tools/dbg_carry.py 3 5
