"""Shared helpers for the -m gpu parity tests (test infrastructure)."""
import numpy as np

import oracle as O
from kcep import native as N


def group_by_key(key, *arrays):
    """Stable sort by key (the host driver's job); returns order + permuted arrays."""
    order = np.argsort(np.asarray(key), kind="stable")
    return order, [None if a is None else np.asarray(a)[order] for a in (key,) + arrays]


def oracle_matches(ir, key, cols, coltypes, mode, **kw):
    p = O.OraclePattern(ir)
    b = O.BatchArrays(key, cols, coltypes, **kw)
    r = O.OracleRun(p, mode)
    r.process(b)
    return [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]


def product_matches(sess: N.Session, out):
    names = sess.pattern.names
    res = []
    for m in range(len(out["match_record"])):
        a, b = out["ent_off"][m], out["ent_off"][m + 1]
        trav = [(names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]
        res.append((int(out["match_record"][m]), int(out["match_key"][m]), trav))
    return res


def run_product(ir, key, cols, mode=N.MODE_PROCESSOR, max_events=None, **kw):
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, max_events or max(1, len(key)), mode=mode)
    s.push(len(key), np.ascontiguousarray(key, np.int32), [np.ascontiguousarray(c) for c in cols], **kw)
    out = s.collect()
    return product_matches(s, out), s
