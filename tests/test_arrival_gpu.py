"""CEP_BATCH_ARRIVAL_ORDER: carry batches handed over in arrival order, as CEPProcessor.process sees its
records one at a time (CEPProcessor.java:134-150).  The library groups each batch by key on the device
(csrc/group.hip) and returns the matches in arrival order of their completing record -- per record in
matchPattern's emission order -- with arrival positions as stream positions.  So the device's output
over a stream cut into batches anywhere must equal the oracle's run over the same interleaved stream,
element by element and in the same order, with no host sort on either side."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import synth
from gpu_util import product_matches
import patterns_lib as PL

pytestmark = pytest.mark.gpu

CASES = [
    ("c2_strict", synth.c2_pattern, 4, N.PATH_STENCIL),
    ("c5_optional", PL.c5_optional, 64, N.PATH_CHAIN),
    ("c3_stock", PL.c3_stock, 7, N.PATH_RUNS),
    ("c4_any", PL.c4_any, 4, N.PATH_GENERAL),
    ("next_one_or_more", PL.next_one_or_more, 4, N.PATH_GENERAL),
    ("any_any", PL.any_any, 4, N.PATH_GENERAL),
]


def oracle_run(ir, key, cols, coltypes, mode=O.MODE_PROCESSOR, **kw):
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    err = None
    try:
        r.process(O.BatchArrays(key, cols, coltypes, **kw))
    except O.OracleError as e:
        err = (e.code, e.record)
    return [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal])
            for m in r.matches(with_groups=False)], err


def stream(name, seed, n_keys, per_key, vmax):
    rng = np.random.default_rng(seed)
    key = np.repeat(np.arange(n_keys, dtype=np.int32), rng.poisson(per_key, n_keys) + 1)
    rng.shuffle(key)                                     # interleaved arrival, like a topic partition
    if name == "c3_stock":
        val = (100 + np.cumsum(rng.integers(-5, 6, len(key)))).astype(np.int32)
    else:
        val = rng.integers(0, vmax, len(key)).astype(np.int32)
    return key, val


def push_arrival(sess, key, cols, bounds, mem="host", **kw):
    import torch
    got, err = [], None
    for a, b in zip(bounds[:-1], bounds[1:]):
        if b == a:
            continue
        kb = np.ascontiguousarray(key[a:b])
        cb = [np.ascontiguousarray(c[a:b]) for c in cols]
        kwb = {k: np.ascontiguousarray(v[a:b]) for k, v in kw.items()}
        if mem == "device":
            t = [torch.from_numpy(x).cuda() for x in [kb] + cb]
            tk = {k: torch.from_numpy(v).cuda() for k, v in kwb.items()}
            torch.cuda.synchronize()
            sess.push(b - a, t[0].data_ptr(), [x.data_ptr() for x in t[1:]], mem=N.MEM_DEVICE,
                      flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE,
                      **{k: v.data_ptr() for k, v in tk.items()})
        else:
            sess.push(b - a, kb, cb, flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE, **kwb)
        out = sess.collect(raise_on_error=False)
        ms = product_matches(sess, out)
        if out["err"]:
            got += [m for m in ms if m[0] < out["err_record"]]
            return got, (int(out["err"]), int(out["err_record"]))
        got += ms
    return got, err


@pytest.mark.parametrize("nbatch", [1, 3, 9])
@pytest.mark.parametrize("name,mk,vmax,path", CASES, ids=[c[0] for c in CASES])
def test_arrival_batches_match_the_reference_in_order(name, mk, vmax, path, nbatch):
    per_key = 8 if name in ("c4_any", "any_any") else 25
    key, val = stream(name, len(name) + nbatch, 150, per_key, vmax)
    ir = mk().to_ir(PL.I32)
    want, oerr = oracle_run(ir, key, [val], [1])
    rng = np.random.default_rng(nbatch)
    bounds = [0] + sorted(rng.choice(np.arange(1, len(key)), nbatch - 1, replace=False).tolist()) + [len(key)]
    sess = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=150, lane_nfa=False)
    assert sess.path == path
    got, gerr = push_arrival(sess, key, [val], bounds)
    assert oerr is None and gerr is None
    assert len(want) > 0 and got == want                 # same matches, same (forward) order


@pytest.mark.parametrize("name,mk,vmax,path", CASES[:3] + CASES[4:5], ids=[c[0] for c in CASES[:3] + CASES[4:5]])
def test_arrival_hot_keys_across_chunks(name, mk, vmax, path):
    """A few hot keys over many 1024-record chunks (the grouping's per-key node lists span chunks) beside
    a thousand cold keys (a chunk's LDS table holds ~1000 distinct keys), device-resident columns."""
    rng = np.random.default_rng(7)
    n = 20000
    key = np.where(rng.random(n) < 0.6, rng.integers(0, 3, n), rng.integers(3, 3000, n)).astype(np.int32)
    if name == "c3_stock":
        val = (100 + np.cumsum(rng.integers(-5, 6, n))).astype(np.int32)
    else:
        val = rng.integers(0, vmax, n).astype(np.int32)
    ir = mk().to_ir(PL.I32)
    want, oerr = oracle_run(ir, key, [val], [1])
    sess = N.Session(N.CompiledPattern(ir), n, carry=True, max_keys=1 << 20, lane_nfa=False)
    assert sess.path == path
    got, gerr = push_arrival(sess, key, [val], [0, 7777, n], mem="device")
    assert oerr is None and gerr is None
    assert len(want) > 0 and got == want


def test_arrival_offsets_topics_and_record_at_a_time():
    """Offsets, timestamps and topics travel with their records through the grouping (the general
    path's high-water marks read them); batches of 1 and 2 records."""
    key, val = stream("next_one_or_more", 5, 40, 10, 4)
    n = len(key)
    off = np.arange(n, dtype=np.int64) * 3 + 11
    ts = np.arange(n, dtype=np.int64) * 1000
    ir = PL.next_one_or_more().to_ir(PL.I32)
    want, _ = oracle_run(ir, key, [val], [1], offset=off, ts=ts)
    for step in (1, 2):
        sess = N.Session(N.CompiledPattern(ir), 4, carry=True, max_keys=40)
        got, err = push_arrival(sess, key, [val], list(range(0, n, step)) + [n], offset=off, ts=ts)
        assert err is None and got == want and len(want) > 0


def test_arrival_exceptions_are_reported_in_arrival_order():
    """The stock demo on random interleaved quotes throws for several keys of one batch: the batch's
    first exception in ARRIVAL order is reported (cep_collect's err_record, cep_batch_errors ascending),
    and the matches before it are the reference's forwards."""
    from kcep import Schema
    sch = Schema([("price", "i64"), ("volume", "i64")])
    rng = np.random.default_rng(17)
    n = 5000
    kid = rng.integers(0, 200, n).astype(np.int32)
    price = (120 + rng.integers(-6, 7, n)).astype(np.int64)
    vol = rng.integers(600, 1200, n).astype(np.int64)
    ir = PL.stock_demo().to_ir(sch)
    want, oerr = oracle_run(ir, kid, [price, vol], [2, 2])
    assert oerr is not None
    sess = N.Session(N.CompiledPattern(ir), n, carry=True, max_keys=200)
    sess.push(n, kid, [price, vol], flags=N.BATCH_ARRIVAL_ORDER)
    out = sess.collect(raise_on_error=False)
    rec, code = sess.batch_errors()
    assert len(rec) > 1 and list(rec) == sorted(rec)
    assert (int(out["err"]), int(out["err_record"])) == (int(code[0]), int(rec[0])) == oerr
    got = [m for m in product_matches(sess, out) if m[0] < out["err_record"]]
    assert got == [m for m in want if m[0] < oerr[1]] and len(got) > 0


@pytest.mark.parametrize("name,mk", [("c2_strict", synth.c2_pattern), ("c3_stock", PL.c3_stock),
                                     ("any_any", PL.any_any)])
def test_arrival_key_out_of_range_is_rejected(name, mk):
    ir = mk().to_ir(PL.I32)
    sess = N.Session(N.CompiledPattern(ir), 8, carry=True, max_keys=4)
    with pytest.raises(N.CepError) as e:
        sess.push(4, np.array([1, 9, 1, 2], np.int32), [np.array([0, 1, 2, 3], np.int32)],
                  flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE)
        sess.collect()
    assert e.value.code == 11
    with pytest.raises(N.CepError) as e:
        N.Session(N.CompiledPattern(ir), 8).push(1, np.array([1], np.int32), [np.array([0], np.int32)],
                                                  flags=N.BATCH_ARRIVAL_ORDER)
    assert e.value.code == 12                           # needs a carry session


def test_arrival_checksum_and_export_speak_arrival_positions():
    """cep_checksum over a stencil carry batch pushed in arrival order equals the oracle's over the
    interleaved stream; a checkpoint (KCSH halo export) taken after it resumes in a fresh session."""
    key, val = stream("c2_strict", 3, 300, 12, 4)
    n = len(key)
    ir = synth.c2_pattern().to_ir(PL.I32)
    want, _ = oracle_run(ir, key, [val], [1])
    s1 = N.Session(N.CompiledPattern(ir), n, carry=True, max_keys=300)
    half = n // 2
    s1.push(half, key[:half], [val[:half]], flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE)
    m1, c1 = s1.checksum()
    got1 = product_matches(s1, s1.collect())
    assert m1 == len(got1) == sum(1 for w in want if w[0] < half)
    s2 = N.Session(N.CompiledPattern(ir), n, carry=True, max_keys=300)
    s2.state_import(s1.state_export())
    s2.push(n - half, np.ascontiguousarray(key[half:]), [np.ascontiguousarray(val[half:])],
            flags=N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE)
    got2 = product_matches(s2, s2.collect())
    assert got1 + got2 == want and len(got2) > 0


@pytest.mark.parametrize("name,mk", [("c2_strict", synth.c2_pattern), ("c5_optional", PL.c5_optional)])
def test_pipelined_flushes_collect_the_batch_before(name, mk):
    """cep_collect_batch: a stencil / chain carry session delivers each batch into one of two host buffers,
    so batch i + 1 is pushed before batch i is collected; the joined output is the unpipelined one."""
    key, val = stream(name, 9, 200, 20, 64 if name == "c5_optional" else 4)
    ir = mk().to_ir(PL.I32)
    want, _ = oracle_run(ir, key, [val], [1])
    sess = N.Session(N.CompiledPattern(ir), 700, carry=True, max_keys=200)
    bounds = list(range(0, len(key), 613)) + [len(key)]
    got, prev = [], None
    flags = N.BATCH_ARRIVAL_ORDER | N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER
    for a, b in zip(bounds[:-1], bounds[1:]):
        sess.push(b - a, np.ascontiguousarray(key[a:b]), [np.ascontiguousarray(val[a:b])], flags=flags)
        if prev is not None:
            got += product_matches(sess, sess.collect(batch_id=prev))
        prev = sess.batch_id()
    import time
    t0 = time.time()
    while not sess.batch_ready(prev) and time.time() - t0 < 10:
        time.sleep(0.001)
    assert sess.batch_ready(prev)
    got += product_matches(sess, sess.collect(batch_id=prev))
    assert got == want and len(want) > 0
    with pytest.raises(N.CepError):                     # only the last batch and the one before it
        sess.collect(batch_id=prev - 2)
