"""Debug aid: chain carry (record-at-a-time) vs the oracle, printing the first differences per key."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kafkastreams-cep_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import test_carry_gpu as T  # noqa: E402
import oracle as O  # noqa: E402
import patterns_lib as PL  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "abc3"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
rng = np.random.default_rng(len(name))
key = rng.integers(0, 5, 600).astype(np.int32)[:n]
val = rng.integers(0, 4, 600).astype(np.int32)[:n]
ir = T.CHAIN_PATTERNS[name](PL.Event.value()).to_ir(PL.I32)
want, _, _ = T.oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
bounds, order = T.batches_of(key, list(range(step, len(key), step)))
got, sess, err = T.run_carry(ir, key[order], [val[order]], bounds, max_keys=5)
got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
print("path", sess.path, "err", err, "got", len(got), "want", len(want))
for k in range(5):
    g = [m for m in got if m[1] == k]
    w = [m for m in want if m[1] == k]
    if g != w:
        idx = [i for i in range(len(key)) if key[i] == k]
        print("key", k, "records", [(i, int(val[i])) for i in idx[:30]])
        print("  got ", g[:8])
        print("  want", w[:8])
