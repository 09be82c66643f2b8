#!/bin/bash
# C4 general path: wave-kernel parity tests, bench (default scratch vs none), per-key allocation profile.
# Usage: tools/gpu_c4.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c4}
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py tests/test_handoff_gpu.py tests/test_seqagg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for sc in default 0 default 0; do
  if [ $sc = default ]; then unset KCEP_WAVE_SCRATCH; else export KCEP_WAVE_SCRATCH=$sc; fi
  timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_${TAG}_$sc.log 2>&1 || { tail -20 gpurun_out/bench_c4_${TAG}_$sc.log; exit 1; }
  echo "scratch=$sc $(tail -1 gpurun_out/bench_c4_${TAG}_$sc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["checksum"], d["roofline"]["kernel_ms"])')"
done
unset KCEP_WAVE_SCRATCH
timeout -k 10 300 python -u tools/c4_profile.py > gpurun_out/c4_profile_$TAG.log 2>&1 || { tail -20 gpurun_out/c4_profile_$TAG.log; exit 1; }
KCEP_WAVE_SCRATCH=0 timeout -k 10 300 python -u tools/c4_profile.py > gpurun_out/c4_profile_${TAG}_noscr.log 2>&1 || { tail -20 gpurun_out/c4_profile_${TAG}_noscr.log; exit 1; }
tail -4 gpurun_out/c4_profile_$TAG.log
tail -4 gpurun_out/c4_profile_${TAG}_noscr.log
echo done
