"""General-path kernel time vs keys per wave (KCEP_NFA_SPREAD) on light keys: the C2 pattern forced
onto the general path.  Usage (GPU box): KCEP_NFA_SPREAD=8 python tools/spread_probe.py N_EVENTS N_KEYS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
import torch  # noqa: E402
from kcep import native as N, synth, Schema  # noqa: E402

n, K = int(sys.argv[1]), int(sys.argv[2])
key, val, order = synth.c2_stream_torch(n, K, "cuda")
cp = N.CompiledPattern(synth.c2_pattern().to_ir(Schema([("value", "i32")])))
s = N.Session(cp, n, force_path=N.PATH_GENERAL)
st = torch.cuda.current_stream().cuda_stream
ms = []
for i in range(4):
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=st)
    ms.append(s.last_kernel_ms())
print(f"spread={os.environ.get('KCEP_NFA_SPREAD', '64')} n={n} keys={K} kernel_ms={min(ms[1:]):.3f} matches={s.checksum()[0]}")
