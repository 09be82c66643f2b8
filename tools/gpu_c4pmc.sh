#!/bin/bash
# C4: bench line, then kcep_nfa_wave's HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, separate passes)
# Usage: tools/gpu_c4pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c4}
export TMPDIR=/tmp
mkdir -p gpurun_out/c4pmc
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --handoff-cap 0 > gpurun_out/c4pmc/b_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/c4pmc/b_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["checksum"], d["first_kernel"])'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/c4pmc/${TAG}_$c -o p -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --carry-batches 1 --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/c4pmc/${TAG}_$c.log 2>&1 || exit 1
done
python3 - gpurun_out/c4pmc/${TAG} <<'PY'
import csv, glob, sys
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = [float(r["Counter_Value"]) * 1024 for f in glob.glob(f"{sys.argv[1]}_{c}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("kcep_nfa_wave")]
    out[c] = sum(v) / len(v) / 1e6
print("kcep_nfa_wave MB per launch: fetch x2 %.1f write %.1f total %.1f" % (2 * out["FETCH_SIZE"], out["WRITE_SIZE"], 2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]))
PY
