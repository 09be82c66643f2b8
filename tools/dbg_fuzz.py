"""Debug one fuzz seed (tests/fuzz_patterns.py) on the GPU: the keys given, one engine option set;
prints the oracle's and the device's error and match counts.  Usage:
python tools/dbg_fuzz.py SEED KEYS(a:b) OPT(jit_wave|interp_lane|interp_wave|jit_lane) [VARIANT mixed|strict|runs]
[MODE 1|2]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "kafkastreams-cep_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import oracle as O
from kcep import native as N
import fuzz_patterns as F, patterns_lib as PL

seed = int(sys.argv[1]); ka, kb = map(int, sys.argv[2].split(":")); opt = sys.argv[3]
variant = sys.argv[4] if len(sys.argv) > 4 else "mixed"
pat, desc, _ = F.pattern_for(seed, variant)
ir = pat.to_ir(PL.I32)
key, val, ts = F.stream_for(seed, variant)
m = (key >= ka) & (key < kb)
key, val, ts = np.ascontiguousarray(key[m]), np.ascontiguousarray(val[m]), np.ascontiguousarray(ts[m])
rng = np.random.default_rng(seed)
omode = O.MODE_PROCESSOR if rng.random() < 0.5 else O.MODE_NFA_PER_KEY
if len(sys.argv) > 5:
    omode = int(sys.argv[5])
gmode = N.MODE_PROCESSOR if omode == O.MODE_PROCESSOR else N.MODE_NFA
p = O.OraclePattern(ir); r = O.OracleRun(p, omode); oerr = None
try:
    r.process(O.BatchArrays(key, [val], [1], ts=ts))
except O.OracleError as e:
    oerr = (e.code, e.record)
print("pattern", desc, "records", len(key), "mode", omode, "oracle", len(r.matches(with_groups=False)), oerr, flush=True)
opts = dict(jit_wave={}, jit_lane=dict(force_path=N.PATH_GENERAL, lane_nfa=True),
            interp_lane=dict(force_path=N.PATH_GENERAL, interpret=True, lane_nfa=True),
            interp_wave=dict(force_path=N.PATH_GENERAL, interpret=True))[opt]
cp = N.CompiledPattern(ir)
s = N.Session(cp, len(key), mode=gmode, **opts)
t = time.time()
s.push(len(key), key, [val], ts=ts)
out = s.collect(raise_on_error=False)
print("device", opt, "path", s.path, "matches", len(out["match_record"]), "err", int(out["err"]), int(out["err_record"]),
      "s", round(time.time() - t, 2), flush=True)
