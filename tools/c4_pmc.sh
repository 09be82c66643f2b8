#!/bin/bash
# SQ instruction / wait counters of the C4 general-path kernel, full batch and the heaviest key alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c4pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/c4pmc -o p1 -- python3 tools/c4_single.py --top1 > gpurun_out/c4pmc/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d gpurun_out/c4pmc -o p2 -- python3 tools/c4_single.py --top1 > gpurun_out/c4pmc/p2.log 2>&1 || exit 1
echo done
