"""Per-dispatch means of rocprofv3 --pmc counters for one kernel, from the counter_collection.csv
files under a directory (one file per pass).  Usage: sq_summary.py DIR KERNEL_SUBSTRING [OUT.json] [NOTE]
SQ_*_CYCLES are in quad-cycles on gfx950; the derived shares are of SQ_WAVE_CYCLES."""
import csv
import glob
import json
import os
import sys

d, kname = sys.argv[1], sys.argv[2]
vals = {}
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    per = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kname not in r["Kernel_Name"]:
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (_, c), v in per.items():
        vals.setdefault(c, []).append(v)
out = {c: sum(v) / len(v) for c, v in sorted(vals.items())}
out["dispatches"] = max((len(v) for v in vals.values()), default=0)
wc = out.get("SQ_WAVE_CYCLES")
if wc:
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in out:
            out[c + "_share"] = out[c] / wc
if out.get("SQ_WAVES"):
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_FLAT",
              "SQ_INSTS_SMEM"):
        if c in out:
            out[c + "_per_wave"] = out[c] / out["SQ_WAVES"]
if len(sys.argv) > 4:
    out["note"] = sys.argv[4]
print(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)
