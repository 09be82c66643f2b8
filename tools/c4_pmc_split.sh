#!/bin/bash
# Where C4's kcep_nfa_wave traffic goes: L1->L2 requests by memory type, L2 write-backs / evictions,
# hits / misses; per workspace placement (KCEP_WAVE_SCRATCH: 0 = pool only, default = scratch regions).
# Usage: tools/c4_pmc_split.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-split}
D=gpurun_out/c4split_$TAG
mkdir -p $D
run() {  # name, scratch, counters...
  local nm=$1 sc=$2; shift 2
  if [ "$sc" = default ]; then unset KCEP_WAVE_SCRATCH; else export KCEP_WAVE_SCRATCH=$sc; fi
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $D -o ${nm}_$sc -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-input --carry-batches 1 --processor-batch , --handoff-cap 0 > $D/${nm}_$sc.log 2>&1 || return 1
  echo "pass $nm scratch=$sc ok"
}
for sc in ${SCRATCH_VARIANTS:-default 0}; do
  run a $sc TCP_TCC_RW_WRITE_REQ_sum TCP_TCC_NC_WRITE_REQ_sum TCP_TCC_UC_WRITE_REQ_sum TCP_TCC_CC_WRITE_REQ_sum || exit 1
  run b $sc TCC_NORMAL_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit 1
  run c $sc TCP_TCC_RW_READ_REQ_sum TCP_TCC_NC_READ_REQ_sum TCP_TCC_UC_READ_REQ_sum TCP_TCC_CC_READ_REQ_sum || exit 1
  run d $sc TCC_HIT_sum TCC_MISS_sum TCC_WRITE_sum TCC_READ_sum || exit 1
  run e $sc SQ_INSTS_FLAT SQ_INSTS_FLAT_NO_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES || exit 1
done
unset KCEP_WAVE_SCRATCH
echo done
