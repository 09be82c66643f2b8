"""Random-pattern parity fuzz (tests/fuzz_patterns.py): each seed builds a pattern through the
reference's builder surface and a key-grouped stream with timestamps, runs it through libkcep.so on
cuda:0 -- once on the path the product picks for it (stencil / chain / runs / general, JIT'd as in
production) and once on the general path forced (interpreted; wave or lane engine by seed) -- and
compares both bit-exactly with oracle/cep_oracle.c: every match (emitting record, key, full buffer
traversal), and the reference's own exception (code and failing record, NFA.java:148-155) where the
pattern raises one, with the matches of the records before it.  The carry variant interleaves the
keys (arrival order, as a topic partition delivers them), cuts the stream into 2-6 batches and runs
them through one carry session (CEP_SESSION_CARRY: each key's state kept on the device between
batches, CEPProcessor.java:111-124), checkpointed at a random batch boundary into a fresh session
(state export / import), against the oracle's single pass over the same records."""
import os

import numpy as np
import pytest

import oracle as O
from kcep import native as N
import fuzz_patterns as F
import patterns_lib as PL

pytestmark = pytest.mark.gpu

# 12 seeds of each variant in the default suite (mostly JIT builds); KCEP_FUZZ_SEEDS=a:b for a campaign
_a, _b = map(int, os.environ.get("KCEP_FUZZ_SEEDS", "0:12").split(":"))
SEEDS = range(_a, _b)


def _oracle(ir, mode, key, val, ts, cols=None, coltypes=(1,), **kw):
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    err = None
    try:
        r.process(O.BatchArrays(key, cols or [val], list(coltypes), ts=ts, **kw))
    except O.OracleError as e:
        err = (e.code, e.record)
    return [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)], err


def _device(ir, gmode, key, val, ts, cols=None, meta=None, **opts):
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, len(key), mode=gmode, **opts)
    s.push(len(key), key, cols or [val], ts=ts, **(meta or {}))
    out = s.collect(raise_on_error=False)
    got, err = [], None
    if out is not None:
        for m in range(len(out["match_record"])):
            a, b = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]))
        if out["err"]:
            err = (int(out["err"]), int(out["err_record"]))
    return got, err, s.path


@pytest.mark.parametrize("variant", ["mixed", "strict", "runs"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_pattern_parity(seed, variant):
    pat, desc, _ = F.pattern_for(seed, variant)
    ir = pat.to_ir(PL.I32)
    try:
        O.OraclePattern(ir)
    except O.OracleError as e:          # an invalid pattern: the product refuses it the same way
        with pytest.raises(N.CepError) as ei:
            N.CompiledPattern(ir)
        assert ei.value.code == e.code
        return
    key, val, ts = F.stream_for(seed, variant)
    rng = np.random.default_rng(seed)
    omode = O.MODE_PROCESSOR if rng.random() < 0.5 else O.MODE_NFA_PER_KEY
    gmode = N.MODE_PROCESSOR if omode == O.MODE_PROCESSOR else N.MODE_NFA
    want, oerr = _oracle(ir, omode, key, val, ts)
    lane = bool(rng.random() < 0.5)
    for opts in (dict(), dict(force_path=N.PATH_GENERAL, interpret=True, lane_nfa=lane)):
        got, gerr, path = _device(ir, gmode, key, val, ts, **opts)
        w = want
        if oerr is not None:             # the task stops at its first exception: earlier records' matches
            got = [m for m in got if m[0] < oerr[1]]
            w = [m for m in want if m[0] < oerr[1]]
        ctx = (seed, desc, omode, path, opts)
        assert gerr == oerr, ctx
        assert got == w, ctx


def _carry_stream(seed, variant):
    """The seed's records in interleaved arrival order, timestamps rising in that order, cut into
    2-6 batches; every batch grouped by key (stable), as the host driver hands it to the device."""
    key, val, _ = F.stream_for(seed, variant)
    rng = np.random.default_rng(seed + 104729)
    perm = rng.permutation(len(key))
    key, val = key[perm], val[perm]
    ts = np.cumsum(rng.integers(1, 4, len(key))).astype(np.int64)
    nb = int(rng.integers(2, 7))
    bounds = [0] + sorted(rng.choice(np.arange(1, len(key)), nb - 1, replace=False).tolist()) + [len(key)]
    order = np.concatenate([a + np.argsort(key[a:b], kind="stable") for a, b in zip(bounds[:-1], bounds[1:])])
    return key[order], val[order], ts[order], bounds


@pytest.mark.parametrize("variant", ["mixed", "strict", "runs"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_pattern_carry_parity(seed, variant):
    pat, desc, _ = F.pattern_for(seed, variant)
    ir = pat.to_ir(PL.I32)
    try:
        O.OraclePattern(ir)
    except O.OracleError:
        pytest.skip("invalid pattern (test_random_pattern_parity checks the refusal)")
    key, val, ts, bounds = _carry_stream(seed, variant)
    rng = np.random.default_rng(seed + 1)
    omode = O.MODE_PROCESSOR if rng.random() < 0.5 else O.MODE_NFA_PER_KEY
    gmode = N.MODE_PROCESSOR if omode == O.MODE_PROCESSOR else N.MODE_NFA
    want, oerr = _oracle(ir, omode, key, val, ts)
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, max(b - a for a, b in zip(bounds[:-1], bounds[1:])), mode=gmode, carry=True,
                  max_keys=int(key.max()) + 1, lane_nfa=bool(rng.random() < 0.5))
    got, gerr = [], None
    ckpt = int(rng.integers(1, len(bounds) - 1))        # checkpoint: restore into a fresh session here
    for j, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        if j == ckpt:                                    # cep_state_export / cep_state_import
            blob = s.state_export()
            s = N.Session(cp, max(b - a for a, b in zip(bounds[:-1], bounds[1:])), mode=gmode, carry=True,
                          max_keys=int(key.max()) + 1, lane_nfa=bool(rng.random() < 0.5))
            s.state_import(blob)
            assert s.stream_position() == a
        s.push(b - a, np.ascontiguousarray(key[a:b]), [np.ascontiguousarray(val[a:b])], ts=np.ascontiguousarray(ts[a:b]))
        out = s.collect(raise_on_error=False)
        for m in range(len(out["match_record"])):
            x, y = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(x, y)]))
        if out["err"]:
            gerr = (int(out["err"]), int(out["err_record"]))
            break
    ctx = (seed, desc, omode, s.path, len(bounds) - 1)
    if oerr is not None:
        got = [m for m in got if m[0] < oerr[1]]
        want = [m for m in want if m[0] < oerr[1]]
    assert gerr == oerr, ctx
    assert got == want, ctx


@pytest.mark.parametrize("seed", SEEDS)
def test_random_rich_parity(seed):
    """The rich variant: i32/i64/f64 columns, stages reading one topic, null records and (processor
    mode) re-delivered records, on the product's path and the forced general path."""
    pat, desc, _ = F.random_pattern(seed, rich=True)
    ir = pat.to_ir(F.RICH)
    try:
        O.OraclePattern(ir)
    except O.OracleError:
        pytest.skip("invalid pattern (test_random_pattern_parity checks the refusal)")
    key, val, ts = F.random_stream(seed)
    rng = np.random.default_rng(seed + 2)
    omode = O.MODE_PROCESSOR if rng.random() < 0.5 else O.MODE_NFA_PER_KEY
    gmode = N.MODE_PROCESSOR if omode == O.MODE_PROCESSOR else N.MODE_NFA
    val, ts, px, r, topic, valid, offset = F.rich_columns(seed, key, val, ts, omode == O.MODE_PROCESSOR)
    cols = [val, px, r]
    meta = dict(topic=topic, valid=valid, offset=offset)
    want, oerr = _oracle(ir, omode, key, val, ts, cols=cols, coltypes=(1, 2, 3), **meta)
    lane = bool(rng.random() < 0.5)
    for opts in (dict(), dict(force_path=N.PATH_GENERAL, interpret=True, lane_nfa=lane)):
        got, gerr, path = _device(ir, gmode, key, val, ts, cols=cols, meta=meta, **opts)
        w = want
        if oerr is not None:
            got = [m for m in got if m[0] < oerr[1]]
            w = [m for m in want if m[0] < oerr[1]]
        ctx = (seed, desc, omode, path, opts)
        assert gerr == oerr, ctx
        assert got == w, ctx


@pytest.mark.parametrize("variant", ["mixed", "strict", "runs"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_pattern_arrival_parity(seed, variant):
    """Processor flushes in arrival order (CEP_BATCH_ARRIVAL_ORDER, csrc/group.hip): the interleaved
    stream cut into 1-6 batches handed over ungrouped; the device groups each batch by key and returns
    the matches in the reference's forward order (CEPProcessor.java:134-150), element by element."""
    pat, desc, _ = F.pattern_for(seed, variant)
    ir = pat.to_ir(PL.I32)
    try:
        O.OraclePattern(ir)
    except O.OracleError:
        pytest.skip("invalid pattern (test_random_pattern_parity checks the refusal)")
    key, val, _ = F.stream_for(seed, variant)
    rng = np.random.default_rng(seed + 3)
    perm = rng.permutation(len(key))
    key, val = np.ascontiguousarray(key[perm]), np.ascontiguousarray(val[perm])
    ts = np.cumsum(rng.integers(1, 4, len(key))).astype(np.int64)
    off = np.arange(len(key), dtype=np.int64)
    nb = int(rng.integers(1, 7))
    bounds = [0] + sorted(rng.choice(np.arange(1, len(key)), nb - 1, replace=False).tolist()) + [len(key)]
    want, oerr = _oracle(ir, O.MODE_PROCESSOR, key, val, ts, offset=off)
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, len(key), carry=True, max_keys=int(key.max()) + 1, lane_nfa=bool(rng.random() < 0.5))
    got, gerr = [], None
    for a, b in zip(bounds[:-1], bounds[1:]):
        s.push(b - a, key[a:b].copy(), [val[a:b].copy()], flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE,
               ts=ts[a:b].copy(), offset=off[a:b].copy())
        out = s.collect(raise_on_error=False)
        for m in range(len(out["match_record"])):
            x, y = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(x, y)]))
        if out["err"]:
            gerr = (int(out["err"]), int(out["err_record"]))
            break
    ctx = (seed, desc, s.path, nb)
    if oerr is not None:
        got = [m for m in got if m[0] < oerr[1]]
        want = [m for m in want if m[0] < oerr[1]]
    assert gerr == oerr, ctx
    assert got == want, ctx


@pytest.mark.parametrize("variant", ["mixed", "runs"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_pattern_evict_to_reference(seed, variant):
    """A key's carried state in the reference's own terms: a general-path carry session in processor
    mode evicts one key at a random batch boundary (cep_state_evict), cep_state_to_reference rewrites
    its state as the reference's stores would hold it (NFAStates.java:33-109, MatchedEvent.java:27-169,
    AggregatesStoreImpl.java:30-76), and the oracle continues that key from it over the key's later
    records while the device continues every other key.  Per key, the joined matches must be the
    uninterrupted reference run's."""
    from test_handoff_gpu import parse_kcrf_events
    pat, desc, _ = F.pattern_for(seed, variant)
    ir = pat.to_ir(PL.I32)
    try:
        O.OraclePattern(ir)
    except O.OracleError:
        pytest.skip("invalid pattern")
    key, val, _ = F.random_stream(seed)
    rng = np.random.default_rng(seed + 5)
    perm = rng.permutation(len(key))
    key, val = np.ascontiguousarray(key[perm]), np.ascontiguousarray(val[perm])
    off = np.arange(len(key), dtype=np.int64)
    ts = off * 2
    full, oerr = _oracle(ir, O.MODE_PROCESSOR, key, val, ts, offset=off)
    if oerr is not None:
        pytest.skip("the reference run raises (the hand-off is checked on exception-free streams)")
    want = {}
    for rec, k, trav in full:
        want.setdefault(k, []).append((rec, trav))
    nb = int(rng.integers(2, 5))
    bounds = [0] + sorted(rng.choice(np.arange(1, len(key)), nb - 1, replace=False).tolist()) + [len(key)]
    cut = bounds[int(rng.integers(1, nb))]
    both = sorted(set(key[:cut].tolist()) & set(key[cut:].tolist()))
    ek = int(rng.choice(both))                           # the evicted key: records on both sides
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, len(key), mode=N.MODE_PROCESSOR, carry=True, max_keys=int(key.max()) + 1,
                  force_path=N.PATH_GENERAL, lane_nfa=bool(rng.random() < 0.5))
    got, pos_rec = {}, {}
    for a, b in zip(bounds[:-1], bounds[1:]):
        if a == cut:                                     # hand the key to the reference
            blob = s.state_evict([ek])[0]
            rest = np.nonzero(key[cut:] == ek)[0] + cut
            if blob:
                ref = cp.state_to_reference(blob)
                _, _, evs = parse_kcrf_events(ref)
            else:
                ref, evs = None, []
            ok = np.array([ek] * (len(evs) + len(rest)), np.int32)
            ov = np.array([e[5][0] for e in evs] + val[rest].tolist(), np.int32)
            oo = np.array([e[3] for e in evs] + off[rest].tolist(), np.int64)
            ot = np.array([e[4] for e in evs] + ts[rest].tolist(), np.int64)
            po = O.OraclePattern(ir)
            r = O.OracleRun(po, O.MODE_PROCESSOR)
            bat = O.BatchArrays(ok, [ov], [1], offset=oo, ts=ot)
            if ref is not None:
                r.resume(bat, ref)
            else:
                r.process(bat)
            for m in r.matches(with_groups=False):    # records named by their offsets = arrival index
                got.setdefault(ek, []).append((int(oo[m.record]), [(po.names[nm], int(oo[e])) for nm, e in m.traversal]))
        idx = np.arange(a, b)
        if a >= cut:
            idx = idx[key[idx] != ek]
        idx = idx[np.argsort(key[idx], kind="stable")]   # grouped by key, arrival order per key
        base = s.stream_position()
        for j, i in enumerate(idx):
            pos_rec[base + j] = int(i)
        s.push(len(idx), key[idx].copy(), [val[idx].copy()], offset=off[idx].copy(), ts=ts[idx].copy(),
               flags=N.BATCH_OFFSETS_MONOTONE)
        out = s.collect(raise_on_error=False)
        assert not out["err"], (seed, desc)
        for m in range(len(out["match_record"])):
            x, y = out["ent_off"][m], out["ent_off"][m + 1]
            got.setdefault(int(out["match_key"][m]), []).append(
                (pos_rec[int(out["match_record"][m])],
                 [(cp.names[out["ent_name"][i]], pos_rec[int(out["ent_record"][i])]) for i in range(x, y)]))
    bad = [k for k in set(got) | set(want) if got.get(k) != want.get(k)]   # (a short message: no list diff)
    assert not bad, (seed, desc, ek, cut, bad[:5], [(len(got.get(k, [])), len(want.get(k, []))) for k in bad[:5]])


@pytest.mark.parametrize("seed", SEEDS)
def test_random_rich_carry_parity(seed):
    """The rich variant as a processor sees a topic partition: interleaved keys, ~5 % null records,
    ~5 % re-deliveries of an earlier record of the same key (same offset and contents, possibly in a
    later batch: the high-water mark carried across batches drops them, CEPProcessor.java:152-160),
    stages reading one topic, i64/f64 predicates; 2-6 carry batches, each grouped by key, against the
    oracle's single pass."""
    pat, desc, _ = F.random_pattern(seed, rich=True)
    ir = pat.to_ir(F.RICH)
    try:
        O.OraclePattern(ir)
    except O.OracleError:
        pytest.skip("invalid pattern")
    key, val, _ = F.random_stream(seed)
    rng = np.random.default_rng(seed + 6)
    perm = rng.permutation(len(key))
    key, val = key[perm], val[perm]
    n = len(key)
    ts = np.cumsum(rng.integers(1, 4, n)).astype(np.int64)
    px = rng.integers(0, 6000, n).astype(np.int64)
    r = rng.random(n)
    topic = rng.integers(0, 2, n).astype(np.int32)
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    off = np.arange(n, dtype=np.int64)
    last = {}
    for i in range(n):                                   # re-delivery: an earlier record of the key again
        k = int(key[i])
        if k in last and rng.random() < 0.05:
            j = int(rng.choice(last[k][-4:]))
            for a in (val, ts, px, r, topic, valid, off):
                a[i] = a[j]
        last.setdefault(k, []).append(i)
    nb = int(rng.integers(2, 7))
    bounds = [0] + sorted(rng.choice(np.arange(1, n), nb - 1, replace=False).tolist()) + [n]
    order = np.concatenate([a + np.argsort(key[a:b], kind="stable") for a, b in zip(bounds[:-1], bounds[1:])])
    key, val, ts, px, r, topic, valid, off = (x[order] for x in (key, val, ts, px, r, topic, valid, off))
    cols = [val, px, r]
    want, oerr = _oracle(ir, O.MODE_PROCESSOR, key, val, ts, cols=cols, coltypes=(1, 2, 3), topic=topic,
                         valid=valid, offset=off)
    cp = N.CompiledPattern(ir)
    mk = lambda **o: N.Session(cp, max(b - a for a, b in zip(bounds[:-1], bounds[1:])), mode=N.MODE_PROCESSOR,
                               carry=True, max_keys=int(key.max()) + 1, lane_nfa=bool(seed & 1), **o)
    s = mk()
    if s.path != N.PATH_GENERAL:
        # the stencil / chain / runs carry sessions carry halos or tails, not per-record processor
        # state: they refuse batches with null records or re-delivered offsets (CEP_E_UNSUPPORTED),
        # and such a stream runs on the general path
        a, b = bounds[0], bounds[1]
        with pytest.raises(N.CepError, match="Unsupported"):
            s.push(b - a, key[a:b].copy(), [c[a:b].copy() for c in cols], ts=ts[a:b].copy(), topic=topic[a:b].copy(),
                   valid=valid[a:b].copy(), offset=off[a:b].copy())
        s = mk(force_path=N.PATH_GENERAL)
    got, gerr = [], None
    for a, b in zip(bounds[:-1], bounds[1:]):
        sl = lambda x: np.ascontiguousarray(x[a:b])
        s.push(b - a, sl(key), [sl(c) for c in cols], ts=sl(ts), topic=sl(topic), valid=sl(valid), offset=sl(off))
        out = s.collect(raise_on_error=False)
        for m in range(len(out["match_record"])):
            x, y = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(x, y)]))
        if out["err"]:
            gerr = (int(out["err"]), int(out["err_record"]))
            break
    ctx = (seed, desc, s.path, nb)
    if oerr is not None:
        got = [m for m in got if m[0] < oerr[1]]
        want = [m for m in want if m[0] < oerr[1]]
    assert gerr == oerr, ctx
    assert got == want, ctx
