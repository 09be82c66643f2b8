"""Summarise one gpu_prof.sh run into profiles/.

usage: python tools/pmc_summary.py TAG_DIR KERNEL EVENTS OUT_PREFIX CONFIG

KERNEL: one kernel, or a comma-separated list whose bytes are summed (a whole step: the runs /
general paths write their CSR in later launches, so their traffic is the step's)

Reads gpurun_out/prof/TAG/{trace_kernel_stats,pmc_fetch_counter_collection,
pmc_write_counter_collection}.csv and writes
  profiles/OUT_PREFIX_kernel_stats.csv   (copy of the rocprofv3 --stats summary)
  profiles/OUT_PREFIX_pmc.json           (per-kernel mean FETCH/WRITE bytes per launch)
  profiles/pmc_traffic[_CONFIG].json     (the bench kernel's HBM bytes per launch; no suffix for c2)

FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE is doubled (gfx950
reports half the bytes of a wide streaming read, MI355X_MICROARCH.md §HBM).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            agg.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag, kernel, events, prefix = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    cfg = sys.argv[5] if len(sys.argv) > 5 else "c2"
    d = os.path.join(ROOT, "gpurun_out", "prof", tag)
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(d, "trace_kernel_stats.csv"), os.path.join(prof, f"{prefix}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(d, "pmc_fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "pmc_write_counter_collection.csv"), "WRITE_SIZE")
    rows = {k: {"fetch_bytes_raw": fetch.get(k), "fetch_bytes_corrected": 2 * fetch[k] if k in fetch else None,
                "write_bytes": write.get(k)} for k in sorted(set(fetch) | set(write))}
    with open(os.path.join(prof, f"{prefix}_pmc.json"), "w") as f:
        json.dump({"tag": tag, "per_launch": rows}, f, indent=1)
    names = kernel.split(",")
    k = {"fetch_bytes_corrected": sum(rows[x]["fetch_bytes_corrected"] or 0 for x in names if x in rows),
         "write_bytes": sum(rows[x]["write_bytes"] or 0 for x in names if x in rows)}
    # the library build the counters were taken on: the bench line of the kernel-trace pass
    build = None
    try:
        with open(os.path.join(ROOT, "gpurun_out", f"prof_trace_{tag}.log")) as f:
            for line in f:
                if line.startswith("{"):
                    build = json.loads(line).get("build", build)
    except OSError:
        pass
    import subprocess
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                            text=True).stdout.strip() or None
    out = {"kernel": kernel, "events": events, "source": f"profiles/{prefix}_pmc.json", "build": build,
           "commit": commit,
           "fetch_bytes_per_launch": k["fetch_bytes_corrected"], "write_bytes_per_launch": k["write_bytes"],
           "hbm_bytes_per_launch": k["fetch_bytes_corrected"] + k["write_bytes"]}
    if len(names) > 1:
        out["kernel"] = "whole cep_push_batch (every kernel of the step, one launch each)"
        out["per_kernel_MB"] = {x: round(((rows[x]["fetch_bytes_corrected"] or 0) + (rows[x]["write_bytes"] or 0)) / 1e6, 1)
                                for x in names if x in rows}
    with open(os.path.join(prof, "pmc_traffic.json" if cfg == "c2" else f"pmc_traffic_{cfg}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
