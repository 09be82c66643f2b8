#!/bin/bash
# general-path parity, then C4 with the cost-ordered schedule vs keys as they come (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_general_gpu.py tests/test_seqagg_gpu.py tests/test_handoff_gpu.py tests/test_processor_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_order.log 2>&1 || { tail -30 gpurun_out/pytest_order.log; exit 1; }
tail -1 gpurun_out/pytest_order.log
for r in 1 2; do
  for v in 1 0; do
    KCEP_NFA_ORDER=$v timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --handoff-cap 0 > gpurun_out/ab/order_${v}_$r.log 2>&1 || { tail -5 gpurun_out/ab/order_${v}_$r.log; exit 1; }
    echo "order=$v run $r $(tail -1 gpurun_out/ab/order_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["checksum"], round(d["first_kernel"]["ms"],3))')"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/ord_c4" -o ord -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --steps 5 --warmup 1 --no-cpu-baseline --handoff-cap 0 > "$GRAFT_REPO_ROOT/gpurun_out/ab/ord_prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import glob, sqlite3
f = glob.glob('gpurun_out/prof/ord_c4/**/*.db', recursive=True)[0]
for r in sqlite3.connect(f).execute("select name, total_calls, average from top_kernels limit 8"):
    print(r[0][:48], r[1], round(r[2] / 1e3, 1))
PY
