import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "kafkastreams-cep_amd")]
import numpy as np
from kcep import native as N, synth, Schema
ir = synth.c2_pattern().to_ir(Schema([("value", "i32")]))
for n in [3, 5, 100, 4096, 4097, 20000, 100000, 1000000]:
    key, val, order = synth.c2_stream_np(n, max(1, n // 100))
    m = np.zeros(n, bool)
    if n >= 3:
        m[2:] = (key[2:] == key[1:-1]) & (key[1:-1] == key[:-2]) & (val[:-2] == 0) & (val[1:-1] == 1) & (val[2:] == 2)
    s = N.Session(N.CompiledPattern(ir), n)
    s.push(n, key, [val])
    out = s.collect()
    print(n, "expected", int(m.sum()), "got", len(out["match_record"]), out["match_record"][:5], np.nonzero(m)[0][:5])
# explicit n=3 ABC
key = np.zeros(3, np.int32); val = np.array([0, 1, 2], np.int32)
s = N.Session(N.CompiledPattern(ir), 3); s.push(3, key, [val]); print("abc", s.collect())
