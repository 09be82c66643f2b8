"""Compile a pattern's per-pattern kernels (cep_pattern_kernel_source) offline with hipcc, as hiprtc
does at run time, and print each kernel's resource usage (VGPRs, SGPRs, scratch, LDS, occupancy).
Usage: jit_isa.py c3|c4|c5 [outdir]  -- writes <outdir>/<cfg>.hip and the ISA <outdir>/<cfg>.s"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
from kcep import native as N, synth, Schema  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "tools", "scratch", "jit")
os.makedirs(out, exist_ok=True)
pat = {"c2": synth.c2_pattern, "c3": synth.c3_pattern, "c4": synth.c4_pattern, "c5": synth.c5_pattern}[cfg]()
cp = N.CompiledPattern(pat.to_ir(Schema([("value", "i32")])))
path = N.PATH_RUNS if cfg == "c3" else N.PATH_GENERAL
src = cp.kernel_source(path)
hip = os.path.join(out, cfg + ".hip")
open(hip, "w").write(src)
csrc = os.path.join(ROOT, "kafkastreams-cep_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-DKCEP_JIT=1",
       "--cuda-device-only", "-S", "-I", csrc, "-I", os.path.join(ROOT, "include"),
       "-Rpass-analysis=kernel-resource-usage", "-o", os.path.join(out, cfg + ".s"), hip]
r = subprocess.run(cmd, capture_output=True, text=True)
for line in r.stderr.splitlines():
    if "remark" in line and ("Function Name" in line or "VGPRs:" in line or "SGPRs" in line or "ScratchSize" in line
                             or "Occupancy" in line or "LDS Size" in line):
        print(line.split("remark: ")[-1])
if r.returncode:
    print(r.stderr[-3000:])
    sys.exit(1)
