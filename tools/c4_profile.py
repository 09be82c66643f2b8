"""Per-key cost profile of the general path on C4 (CEP_SESSION_PROFILE): where the kernel's time goes.

Prints the kernel time, the distribution of per-key cycles / live runs / run evaluations, and the
heaviest keys.  Usage (GPU box): python tools/c4_profile.py [n_keys] [--interpret]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
import torch  # noqa: E402
from kcep import native as N, synth, Schema  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100_000
interp = "--interpret" in sys.argv
key, val, ts = synth.c4_stream_torch(K, "cuda")
n = key.numel()
cp = N.CompiledPattern(synth.c4_pattern().to_ir(Schema([("value", "i32")])))
s = N.Session(cp, n, force_path=N.PATH_GENERAL, profile=True, interpret=interp)
st = torch.cuda.current_stream().cuda_stream
for i in range(3):
    s.push(n, key.data_ptr(), [val.data_ptr()], ts=ts.data_ptr(), mem=N.MEM_DEVICE, stream=st)
    kms = s.last_kernel_ms()
prof = s.key_profile()
if "--save" in sys.argv:                              # per-key rows for offline analysis
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "c4_key_profile.npy"), prof)
cyc = prof[:, 3].astype(np.float64) / 100.0   # wall clock 100 MHz -> us
live, ev = prof[:, 1], prof[:, 2]
print(f"jit={s.jit} kernel {kms:.2f} ms  keys {len(prof)}  live-run hwm {s.live_run_hwm()}")
for nm, a in (("key us", cyc), ("live runs", live), ("evaluations", ev)):
    print(f"{nm:12s} mean {a.mean():9.2f} p50 {np.median(a):9.2f} p99 {np.percentile(a, 99):9.2f} "
          f"p99.9 {np.percentile(a, 99.9):9.2f} max {a.max():9.2f} sum {a.sum():.3e}")
o = np.argsort(-cyc)[:10]
print("heaviest keys (key, live max, evals, us):")
for i in o:
    print("  ", int(prof[i, 0]), int(live[i]), int(ev[i]), round(float(cyc[i]), 1))
print("us per evaluation (top 100 keys):", float(cyc[o[:100]].sum() / max(1, ev[np.argsort(-cyc)[:100]].sum())))
print("corr(evals, us)", float(np.corrcoef(ev, cyc)[0, 1]))
ws = prof[:, 16]
print("workspace words: mean %.0f p50 %.0f p90 %.0f p99 %.0f max %d; heaviest key %d" %
      (ws.mean(), np.median(ws), np.percentile(ws, 90), np.percentile(ws, 99), ws.max(), ws[o[0]]))
ph = prof[:, 4:15].astype(np.float64)
if (ph >= 0).all() and "--wave-phases" in sys.argv:   # the wave kernel's record loop (nfa_wave.h KWP_*)
    names = ["nodes init", "evaluation", "commit", "placement scans", "matchConstruction", "admit+ignored",
             "event-only preds", "round prologue", "record end (incl. matchConstruction)", "-", "placement writes"]
    tot = ph.sum(axis=0)
    full = cyc.sum() * 1e-6 * 2.1e9 / 1e0                  # (shader clocks ~ 2.1 GHz; for scale only)
    print("wave record-loop clocks (sum over keys):", {nm: f"{t:.3e}" for nm, t in zip(names, tot)})
    den = tot[[0, 1, 2, 3, 5, 6, 7, 8, 10]].sum()
    print("shares:", {nm: round(float(t / den), 3) for nm, t in zip(names, tot) if nm != "-"})
elif (ph >= 0).all():
    tot = ph.sum(axis=0)
    print("phase clock sums:", [f"{x:.3e}" for x in tot[:8]], "share:",
          [round(float(x / max(1.0, tot[:5].sum())), 3) for x in tot[:5]])
    names = ["evaluate", "predicates", "buffer put+branch", "removePattern", "matchConstruction", "scans",
             "add_pred", "versions"]
    for sel, nm in ((slice(None), "all keys"), (o[:100], "top-100 keys")):
        tot = ph[sel].sum(axis=0)
        print(nm, "clock share of evaluate+remove+emit:",
              {n: round(float(t / (tot[0] + tot[3] + tot[4])), 3) for n, t in zip(names, tot[:8])})
        print(nm, "scans", int(tot[8]), "entries/scan", round(float(tot[9] / max(1, tot[8])), 2),
              "digit checks/scan", round(float(tot[10] / max(1, tot[8])), 2),
              "clocks/scan", round(float(tot[5] / max(1, tot[8])), 1))
t0 = prof[:, 15].astype(np.float64)
if (t0 > 0).all():                                     # the grid's busy timeline: keys in flight over time
    t1 = t0 + prof[:, 3]
    lo, hi = t0.min(), t1.max()
    ev_t = np.concatenate([t0, t1]); ev_d = np.concatenate([np.ones(len(t0)), -np.ones(len(t1))])
    o2 = np.argsort(ev_t, kind="stable")
    inflight = np.cumsum(ev_d[o2]); tt = ev_t[o2]
    full = inflight.max()
    busy = np.sum(inflight[:-1] * np.diff(tt)) / (full * (hi - lo))
    below = tt[np.nonzero(inflight < 0.9 * full)[0]]
    tail_start = below[below > lo + 0.5 * (hi - lo)].min() if (below > lo + 0.5 * (hi - lo)).any() else hi
    print(f"timeline: span {(hi - lo) / 100:.0f} us, keys in flight max {int(full)}, mean occupancy {busy:.3f}, "
          f"tail (<90% in flight) {(hi - tail_start) / 100:.0f} us; last key starts {(t0.max() - lo) / 100:.0f} us")
    late = np.argsort(-t1)[:5]
    print("  last to finish (key, start us, us):",
          [(int(prof[i, 0]), round((t0[i] - lo) / 100, 1), round(float(cyc[i]), 1)) for i in late])
kinds = ["first workspace", "match output", "heap", "run queues", "private lists", "aggregates", "other"]
kw = prof[:, 17:25].astype(np.float64)
if (kw >= 0).all():
    tot = kw.sum(axis=0)
    print("allocated words per kind over the batch (share):",
          {k: f"{t:.3e} ({t / max(1.0, tot[:7].sum()):.3f})" for k, t in zip(kinds, tot[:7])})
    print(f"  of which from the batch pool: {tot[7]:.3e} words ({tot[7] * 4 / 1e6:.1f} MB); "
          f"from the waves' scratch regions: {tot[:7].sum() - tot[7]:.3e} words")
