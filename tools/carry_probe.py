"""Where a carry stream's time goes: the same device-resident C2 / C5 stream as
  (a) one resident batch, (b) 10 batches on a plain session, (c) 10 batches on a carry session,
with per-push kernel times (HIP events) and wall time per pass.  Usage: carry_probe.py [c2|c5] [batches]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
import torch  # noqa: E402
from kcep import native as N, synth, Schema  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
I32 = Schema([("value", "i32")])
if cfg == "c2":
    K = 1_000_000
    key, val, _ = synth.c2_stream_torch(100_000_000, K, dev)
    ir = synth.c2_pattern().to_ir(I32)
else:
    K = 1_250_000
    key, val, _ = synth.c5_stream_torch(K, dev, L=100)
    ir = synth.c5_pattern().to_ir(I32)
n = key.numel()
st = torch.cuda.current_stream(dev)
pat = N.CompiledPattern(ir)
per = -(-(-(-n // nb)) // 4096) * 4096
bounds = list(range(0, n, per)) + [n]


def run(sess, bnds, timing):
    sess.set_timing(timing)
    ks = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in zip(bnds[:-1], bnds[1:]):
        sess.push(b - a, key.data_ptr() + 4 * a, [val.data_ptr() + 4 * a], mem=N.MEM_DEVICE, stream=st.cuda_stream)
        if timing:
            ks.append(sess.last_kernel_ms())
    st.synchronize()
    return (time.perf_counter() - t0) * 1e3, sum(ks)


for label, carry, bnds in (("resident 1 batch", False, [0, n]), (f"plain {nb} batches", False, bounds),
                           (f"carry {nb} batches", True, bounds)):
    s = N.Session(pat, max(b - a for a, b in zip(bnds[:-1], bnds[1:])), carry=carry, max_keys=K if carry else 0)
    run(s, bnds, False)
    walls, kern = [], []
    for _ in range(5):
        if carry:
            s.state_clear()
        walls.append(run(s, bnds, False)[0])
    for _ in range(3):
        if carry:
            s.state_clear()
        kern.append(run(s, bnds, True)[1])
    print(f"{cfg} {label:18s} wall {min(walls):8.3f} ms   kernels {min(kern):8.3f} ms  (n={n})", flush=True)
