"""Debug: stencil carry record-at-a-time (k=2) on the plain and keyed kernels against the oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kafkastreams-cep_amd"))
import test_carry_gpu as T
from kcep import native as N
import oracle as O
k = int(sys.argv[1]) if len(sys.argv) > 1 else 2
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rng = np.random.default_rng(k)
key = rng.integers(0, 7, 400).astype(np.int32)
val = rng.integers(0, 2, 400).astype(np.int32)
ir = T._strict_pattern(k)
want, _, _ = T.oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
bounds, order = T.batches_of(key, list(range(step, len(key), step)))
got, sess, err = T.run_carry(ir, key[order], [val[order]], bounds, max_keys=7)
got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
print("keyed" if os.environ.get("KCEP_STENCIL_KEYED") else "plain", "err", err, "n got", len(got), "n want", len(want))
sg, sw = sorted(got), sorted(want)
print("first got ", sg[:6])
print("first want", sw[:6])
print("keys", key[:40].tolist())
print("vals", val[:40].tolist())
