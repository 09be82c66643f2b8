#!/bin/bash
# A/B of one build under two environment settings, alternating runs on one box.
# Usage: tools/ab_env.sh TAG CONFIG "ENV_A" "ENV_B" [rounds] [extra bench args]
#   e.g. tools/ab_env.sh stencil_wave c2 "KCEP_STENCIL=wg" "KCEP_STENCIL=wave" 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
TAG=$1; C=$2; A=$3; B=$4; R=${5:-3}; shift 5; EXTRA="$@"
for i in $(seq 1 $R); do
  env $A timeout -k 10 200 python -u bench.py --config $C --steps 50 --warmup 5 --no-cpu-baseline --no-host-input $EXTRA > gpurun_out/ab/${TAG}_a_$i.log 2>&1 || { tail -5 gpurun_out/ab/${TAG}_a_$i.log; exit 1; }
  env $B timeout -k 10 200 python -u bench.py --config $C --steps 50 --warmup 5 --no-cpu-baseline --no-host-input $EXTRA > gpurun_out/ab/${TAG}_b_$i.log 2>&1 || { tail -5 gpurun_out/ab/${TAG}_b_$i.log; exit 1; }
  python3 - "$TAG" "$i" <<'EOF'
import json, sys
tag, i = sys.argv[1], sys.argv[2]
for ab in "ab":
    line = open(f"gpurun_out/ab/{tag}_{ab}_{i}.log").read().strip().splitlines()[-1]
    d = json.loads(line)
    r = d.get("roofline", {})
    print(f"{tag} round {i} {ab}: step {d['ms_per_step']*1e3:.1f} us  kernel {r.get('kernel_ms', 0)*1e3:.1f} us  "
          f"value {d['value']:.4g}  checksum {d.get('checksum')}  carry {d.get('carry_stream', {}).get('ms_per_pass')}")
EOF
done
