"""Is the C4 general-path kernel bound by one key's serial chain, or by contention?

Profiles the full C4 batch, then re-runs only the heaviest keys (by run evaluations) on an
otherwise idle GPU and prints their kernel time.  Usage (GPU box): python tools/c4_single.py [--top1]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
import torch  # noqa: E402
from kcep import native as N, synth, Schema  # noqa: E402

K, L = 100_000, 12
key, val, ts = synth.c4_stream_torch(K, "cuda")
n = key.numel()
cp = N.CompiledPattern(synth.c4_pattern().to_ir(Schema([("value", "i32")])))
st = torch.cuda.current_stream().cuda_stream


def run(k, v, t, profile=False, reps=3):
    s = N.Session(cp, k.numel(), force_path=N.PATH_GENERAL, profile=profile)
    for _ in range(reps):
        s.push(k.numel(), k.data_ptr(), [v.data_ptr()], ts=t.data_ptr(), mem=N.MEM_DEVICE, stream=st)
        ms = s.last_kernel_ms()
    return s, ms


s, ms = run(key, val, ts, profile=True)
prof = s.key_profile()
ev = prof[:, 2]
print(f"full batch: kernel {ms:.2f} ms, max evals {ev.max()}, live hwm {s.live_run_hwm()}", flush=True)
order = np.argsort(-ev)
for top in ((1,) if "--top1" in sys.argv else (1, 8, 64, 1024)):
    ks = np.sort(prof[order[:top], 0])
    idx = torch.as_tensor((ks[:, None] * L + np.arange(L)[None, :]).reshape(-1), device="cuda")
    k2, v2, t2 = key[idx].contiguous(), val[idx].contiguous(), ts[idx].contiguous()
    _, ms2 = run(k2, v2, t2)
    s3, _ = run(k2, v2, t2, profile=True, reps=1)
    p3 = s3.key_profile()
    print(f"top {top:5d} keys alone: kernel {ms2:.3f} ms, max evals {p3[:, 2].max()}, "
          f"max key us {p3[:, 3].max() / 100:.1f}, us/eval of heaviest {p3[:, 3].max() / 100 / max(1, p3[:, 2].max()):.2f}",
          flush=True)
