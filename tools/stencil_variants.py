"""Time the C2 stencil kernel of every build under build_variants/ (HIP events, median)."""
import glob, json, os, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, statistics
sys.path.insert(0, os.path.join(%r, "kafkastreams-cep_amd"))
import torch
from kcep import native as N, synth, Schema
n, K = 100_000_000, 1_000_000
key, val, _ = synth.c2_stream_torch(n, K, "cuda")
torch.cuda.synchronize()
s = N.Session(N.CompiledPattern(synth.c2_pattern().to_ir(Schema([("value", "i32")]))), n)
st = torch.cuda.current_stream().cuda_stream
ms, bms = [], []
for i in range(25):
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=st)
    ms.append(s.last_kernel_ms())
    bms.append(s.last_batch_ms())
nm, cs = s.checksum()
print(json.dumps({"lib": os.environ["KCEP_LIB"], "ms": statistics.median(ms[5:]), "batch_ms": statistics.median(bms[5:]),
                  "matches": nm, "csum": "%%016x" %% cs}))
''' % ROOT
for lib in sorted(glob.glob(os.path.join(ROOT, "build_variants", "*", "libkcep.so"))):
    env = dict(os.environ, KCEP_LIB=lib)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print(out.stdout.strip() or out.stderr[-500:], flush=True)
