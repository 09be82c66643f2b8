#!/bin/bash
# C4 wave kernel: LDS arena words x waves per SIMD (KCEP_WAVE_ARENA, KCEP_NFA_WAVE_OCC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for occ in 3 4; do
  for a in 1024 1536 2048; do
    KCEP_WAVE_ARENA=$a KCEP_NFA_WAVE_OCC=$occ timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c4a_${occ}_$a.log 2>&1 || exit 1
    echo "occ $occ arena $a: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4a_${occ}_$a.log) $(grep -o '"checksum": "[0-9a-f]*"' gpurun_out/c4a_${occ}_$a.log)"
  done
done
