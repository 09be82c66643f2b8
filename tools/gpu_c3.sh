#!/bin/bash
# C3 iteration: runs-path tests, the C3 bench line, a kernel trace.  Usage: tools/gpu_c3.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c3}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_runs_gpu.py tests/test_baseline_sizes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c3_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_c3_$TAG.log
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c3_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c3_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); cs=d.get("carry_stream") or {}; print(round(d["ms_per_step"],4), d["checksum"], d["first_kernel"], "carry", cs.get("ms_per_pass"), cs.get("vs_resident"), cs.get("parity"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/${TAG}_c3 -o trace -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/prof_trace_${TAG}_c3.log 2>&1 || exit 1
python3 - "$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/prof/{sys.argv[1]}_c3/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Name"][:50], r["Calls"], r["AverageNs"])
PY
