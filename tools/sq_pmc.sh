#!/bin/bash
# SQ instruction / wait counters of bench.py's dominant kernel for one config.
# Usage: tools/sq_pmc.sh c5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
C=${1:-c5}
D=gpurun_out/sqpmc_$C
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $D -o p1 -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-input --carry-batches 1 --handoff-cap 0 > $D/p1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT SQ_INSTS_SMEM --output-format csv -d $D -o p2 -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-input --carry-batches 1 --handoff-cap 0 > $D/p2.log 2>&1 || exit 1
echo done
