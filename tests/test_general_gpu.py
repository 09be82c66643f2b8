"""Parity of the general HIP NFA path (csrc/nfa.hip) with the CPU oracle.

Every reference golden scenario and randomized streams for the BASELINE
configs C3-C5 (plus skip-till-next / skip-till-any shapes) are run through
libkcep.so on cuda:0 with the general path forced, and compared bit-exactly
(emitting record, key, full buffer traversal) with oracle/cep_oracle.c on the
same key-grouped batch."""
import zlib

import numpy as np
import pytest

import oracle as O
from kcep import native as N
from golden_util import scenarios, event_arrays, seq_repr
from gpu_util import oracle_matches, product_matches
import patterns_lib as PL

pytestmark = pytest.mark.gpu


def grouped(fx):
    a = event_arrays(fx)
    key = a["key"] if fx["mode"] == O.MODE_PROCESSOR else np.zeros_like(a["key"])
    order = np.argsort(key, kind="stable")
    out = dict(key=key[order], cols=[c[order] for c in a["cols"]], coltypes=a["coltypes"])
    for f in ("topic", "partition", "offset", "ts", "valid"):
        out[f] = None if a[f] is None else a[f][order]
    return out, order


def run_both(ir, mode, key, cols, coltypes, force=N.PATH_GENERAL, interpret=False, lane_nfa=False, **kw):
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    oerr = None
    try:
        r.process(O.BatchArrays(key, cols, coltypes, **kw))
    except O.OracleError as e:
        oerr = (e.code, e.record)
    want = [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, max(1, len(key)), mode=mode, force_path=force, interpret=interpret, lane_nfa=lane_nfa)
    if force == N.PATH_GENERAL:
        assert s.jit == (not interpret)       # kernel compiled for the pattern unless asked otherwise
    s.push(len(key), np.ascontiguousarray(key, np.int32), [np.ascontiguousarray(c) for c in cols], **kw)
    gerr = None
    out = s.collect(raise_on_error=False)
    got = []
    if out is not None:
        for m in range(len(out["match_record"])):
            a, b = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]))
        if out["err"]:
            gerr = (int(out["err"]), int(out["err_record"]))
    if oerr is not None:
        # the reference stops the task at its first exception; the oracle walks the
        # key-grouped batch in order, so the matches forwarded are exactly those of earlier
        # records (matchPattern throws before returning the failing record's list, NFA.java:148-155)
        got = [m for m in got if m[0] < oerr[1]]
        want = [m for m in want if m[0] < oerr[1]]
    return want, got, oerr, gerr


SC = scenarios()


def stable_seed(name, mod):
    """A seed from the case name that is the same in every process (Python's str hash is salted per
    process, so a failure seeded by it could not be reproduced)."""
    return zlib.crc32(name.encode()) % mod


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("fx", SC, ids=[f["name"] for f in SC])
def test_golden_general(fx, interpret, lane_nfa):
    g, order = grouped(fx)
    kw = {k: g[k] for k in ("topic", "partition", "offset", "ts", "valid") if g[k] is not None}
    want, got, oerr, gerr = run_both(bytes.fromhex(fx["ir"]), fx["mode"], g["key"], g["cols"], g["coltypes"],
                                     interpret=interpret, lane_nfa=lane_nfa, **kw)
    assert oerr is None and gerr is None
    assert got == want
    # and the reference's own expectation, compared directly: each device sequence as its stage
    # groups (first-seen stage order reversed, Sequence.Builder.build(true)) of fixture records
    exp = [[(gr["stage"], sorted(gr["events"])) for gr in sq] for sq in fx["expected"]["sequences"]]
    assert sorted(map(repr, device_sequences(got, order))) == sorted(map(repr, exp))


def device_sequences(got, order):
    out = []
    for _rec, _key, trav in got:
        groups, seen = {}, []
        for nm, r in trav:
            if nm not in groups:
                groups[nm] = set()
                seen.append(nm)
            groups[nm].add(int(order[r]))
        out.append([(nm, sorted(groups[nm])) for nm in reversed(seen)])
    return out


def rand_stream(seed, n_keys, per_key, vmax, grouped_keys=True):
    rng = np.random.default_rng(seed)
    lens = rng.poisson(per_key, n_keys) + 1
    key = np.repeat(np.arange(n_keys, dtype=np.int32), lens)
    val = rng.integers(0, vmax, len(key)).astype(np.int32)
    return key, val


CASES = [
    ("c3_stock", PL.c3_stock, 7, lambda rng, n: (100 + np.cumsum(rng.integers(-5, 6, n))).astype(np.int32)),
    ("c4_any", PL.c4_any, 4, None),
    ("c5_optional", PL.c5_optional, 64, None),
    ("next_one_or_more", PL.next_one_or_more, 4, None),
    ("any_any", PL.any_any, 4, None),
]


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("mode", [O.MODE_PROCESSOR, O.MODE_NFA_PER_KEY])
@pytest.mark.parametrize("name,mk,vmax,gen", CASES, ids=[c[0] for c in CASES])
def test_random_general(name, mk, vmax, gen, mode, interpret, lane_nfa):
    per_key = 8 if name in ("c4_any", "any_any") else 30
    key, val = rand_stream(stable_seed(name, 1000), 300, per_key, vmax)
    if gen is not None:
        val = gen(np.random.default_rng(5), len(key))
    ir = mk().to_ir(PL.I32)
    gmode = N.MODE_PROCESSOR if mode == O.MODE_PROCESSOR else N.MODE_NFA
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    r.process(O.BatchArrays(key, [val], [1]))
    want = [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, len(key), mode=gmode, force_path=N.PATH_GENERAL, interpret=interpret, lane_nfa=lane_nfa)
    assert s.jit == (not interpret)
    s.push(len(key), key, [val])
    out = s.collect()
    got = []
    for m in range(len(out["match_record"])):
        a, b = out["ent_off"][m], out["ent_off"][m + 1]
        got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                    [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]))
    assert len(want) > 0
    assert got == want


@pytest.mark.parametrize("seed", [11, 17, 28])
def test_stock_demo_random(seed):
    """The example pattern on random quotes. The reference's buffer deletes nodes that a
    later traversal still reaches, so on random data it throws (NPE at
    SharedVersionedBufferStoreImpl.java:186, or IllegalStateException at :113-115); the
    device path must raise the same exception at the same record, after the same matches."""
    rng = np.random.default_rng(seed)
    key, _ = rand_stream(seed, 200, 25, 4)
    n = len(key)
    price = (120 + rng.integers(-6, 7, n)).astype(np.int64)
    vol = rng.integers(600, 1200, n).astype(np.int64)
    want, got, oerr, gerr = run_both(PL.stock_demo().to_ir(PL.STOCK_SCHEMA), O.MODE_PROCESSOR, key, [price, vol], [2, 2])
    assert oerr is not None and gerr == oerr
    assert got == want


def test_stock_demo_minimal_npe():
    """Smallest input that makes the reference throw: (price, volume) =
    (100,1001) (102,1001) (102,700) (100,500) -> NPE while emitting at record 3."""
    key = np.zeros(4, np.int32)
    price = np.array([100, 102, 102, 100], np.int64)
    vol = np.array([1001, 1001, 700, 500], np.int64)
    want, got, oerr, gerr = run_both(PL.stock_demo().to_ir(PL.STOCK_SCHEMA), O.MODE_PROCESSOR, key, [price, vol], [2, 2])
    assert oerr == (4, 3) and gerr == oerr and got == want


def test_c2_general_matches_stencil():
    from kcep import synth
    key, val, order = synth.c2_stream_np(200_000, 5_000)
    ir = synth.c2_pattern().to_ir(PL.I32)
    want, got, _, _ = run_both(ir, O.MODE_PROCESSOR, key, [val], [1], offset=order, ts=order)
    assert got == want and len(got) > 1000


def test_unknown_aggregate_error_record():
    """States.get on an unset state raises UnknownAggregateException at the same record."""
    from kcep import QueryBuilder, Event, States
    p = (QueryBuilder().select("a").where(Event.value() == 0).then()
         .select("b").where(States.getInt("nope") > 0).build())
    key, val = rand_stream(9, 50, 10, 3)
    want, got, oerr, gerr = run_both(p.to_ir(PL.I32), O.MODE_PROCESSOR, key, [val], [1])
    assert oerr is not None and gerr == oerr


def test_null_records_and_high_water_mark():
    """Processor rules on the general path: null records skipped, re-delivered offsets dropped."""
    rng = np.random.default_rng(4)
    key, val = rand_stream(21, 100, 20, 4)
    n = len(key)
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    offset = np.arange(n, dtype=np.int64)
    dup = rng.random(n) < 0.1
    offset[dup] = np.maximum(offset[dup] - 3, 0)              # re-delivery of older offsets
    ir = PL.any_any().to_ir(PL.I32)
    want, got, oerr, gerr = run_both(ir, O.MODE_PROCESSOR, key, [val], [1], valid=valid, offset=offset)
    assert oerr is None and gerr is None and got == want and len(got) > 0


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
def test_over_capacity_key_is_handed_back_alone(lane_nfa):
    """a key whose runs outgrow the device capacity falls back per key.  With a small
    per-key workspace cap (cep_opts.max_key_words) the exploding skip-till-any key stops at the record
    where it ran out and is listed by cep_batch_errors with CEP_E_RUN_CAPACITY; its matches before
    that record and every other key's matches equal the oracle's, and the batch itself succeeds."""
    rng = np.random.default_rng(4)
    lens = [12] * 40
    lens[7] = 400                                          # the exploding key
    key = np.repeat(np.arange(40, dtype=np.int32), lens)
    val = rng.integers(0, 4, len(key)).astype(np.int32)
    ir = PL.any_any().to_ir(PL.I32)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), len(key), force_path=N.PATH_GENERAL, max_key_words=1 << 17,
                  lane_nfa=lane_nfa)
    s.push(len(key), key, [val])
    out = s.collect(raise_on_error=False)
    rec, code = s.batch_errors()
    assert list(code) == [9] and key[rec[0]] == 7
    got = product_matches(s, out)
    assert got == [m for m in want if m[1] != 7 or m[0] < rec[0]]
    assert any(m[1] == 7 for m in got) and any(m[1] == 7 and m[0] >= rec[0] for m in want)


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
def test_key_over_capacity_at_first_allocation(lane_nfa):
    """A key whose very first workspace allocation is already over cep_opts.max_key_words (5000
    records against 1<<17 words) must still be listed by cep_batch_errors with CEP_E_RUN_CAPACITY
    at its first record -- key_begin raises the batch's error flag, so the host reads the per-key
    errors -- while every other key matches the oracle.  (The strict A->B->C pattern on the general
    path: a long key is cheap for the oracle.)"""
    from kcep import synth
    rng = np.random.default_rng(5)
    lens = [12] * 40
    lens[7] = 5000
    key = np.repeat(np.arange(40, dtype=np.int32), lens)
    val = rng.integers(0, 4, len(key)).astype(np.int32)
    ir = synth.c2_pattern().to_ir(PL.I32)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), len(key), force_path=N.PATH_GENERAL, max_key_words=1 << 17,
                  lane_nfa=lane_nfa)
    s.push(len(key), key, [val])
    out = s.collect(raise_on_error=False)
    rec, code = s.batch_errors()
    first7 = int(np.searchsorted(key, 7))
    assert list(code) == [9] and list(rec) == [first7]
    assert out["err"] == 9
    got = product_matches(s, out)
    assert got == [m for m in want if m[1] != 7]


@pytest.mark.parametrize("order", ["cost", "arrival"])
@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
def test_c4_heavy_keys(lane_nfa, order, monkeypatch):
    """C4 (skip-till-any times(3) + zeroOrMore) keys long enough that one record's run queue holds
    several rounds of 64 runs on the wave kernel; every match, in order, as the oracle's.  The wave
    kernel takes the keys heaviest-estimated first (nfa_dev.h seg_bucket) or as they come
    (KCEP_NFA_ORDER=0): the schedule changes nothing in the output."""
    monkeypatch.setenv("KCEP_NFA_ORDER", "1" if order == "cost" else "0")
    from kcep import synth
    key, val, _ = synth.c4_stream_np(400, L=16)
    ir = synth.c4_pattern().to_ir(PL.I32)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), len(key), force_path=N.PATH_GENERAL, lane_nfa=lane_nfa)
    s.push(len(key), key, [val])
    got = product_matches(s, s.collect())
    assert got == want and len(want) > 0
    assert s.live_run_hwm() > 128


@pytest.mark.parametrize("scratch", ["0", "64", None], ids=["pool_only", "scratch_64", "scratch_default"])
@pytest.mark.parametrize("name,mk,vmax,gen", CASES, ids=[c[0] for c in CASES])
def test_wave_scratch_regions(name, mk, vmax, gen, scratch, monkeypatch):
    """The persistent wave kernel's workspace placement (nfa_wave.h, nfa_dev.h KeyAlloc): keys of every
    size in one batch, each wave recycling its scratch region from key to key, with no region (every
    array that leaves the LDS arena from the batch pool), a 64-word region (keys overflow into the
    pool mid-key) and the default one -- against the oracle."""
    if scratch is None:
        monkeypatch.delenv("KCEP_WAVE_SCRATCH", raising=False)
    else:
        monkeypatch.setenv("KCEP_WAVE_SCRATCH", scratch)
    rng = np.random.default_rng(stable_seed(name, 977))
    if name in ("c4_any", "any_any"):       # skip-till-any: live runs multiply with every record (Q6)
        lens = np.concatenate([rng.integers(1, 6, 200), rng.integers(10, 15, 60)])
    else:
        lens = np.concatenate([rng.integers(1, 6, 200), rng.integers(20, 40, 40), [60, 80]])
    rng.shuffle(lens)
    key = np.repeat(np.arange(len(lens), dtype=np.int32), lens)
    val = (gen(rng, len(key)) if gen is not None else rng.integers(0, vmax, len(key))).astype(np.int32)
    ir = mk().to_ir(PL.I32)
    want, got, oerr, gerr = run_both(ir, O.MODE_PROCESSOR, key, [val], [1], lane_nfa=False)
    assert gerr == oerr
    assert got == want and len(want) > 0


def test_pool_regrowth_is_bounded_and_given_back(monkeypatch):
    """The general path's workspace pool: a batch that overflows it is re-run on a larger
    pool; the next batches start from the grown size (one attempt each, no re-run per batch), and after
    4 batches in a row that fit the estimate the grown pool is given back, so one heavy stretch does not
    hold the device for the session's lifetime; with a budget (cep_opts.max_pool_bytes) the pool stops
    growing there and the keys still out of room are handed back per key (CEP_E_RUN_CAPACITY) while
    every other key completes as the oracle's."""
    import torch
    from kcep import synth
    monkeypatch.setenv("KCEP_WAVE_SCRATCH", "0")          # every workspace array from the pool
    key, val, _ = synth.c4_stream_np(400, L=16)
    ir = synth.c4_pattern().to_ir(PL.I32)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), 2 * len(key), force_path=N.PATH_GENERAL, lane_nfa=False)
    light_k, light_v = key[key < 8], val[key < 8]
    light_want = oracle_matches(ir, light_k, [light_v], [1], O.MODE_PROCESSOR)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    s.push(len(key), key, [val])                           # ~2.1 M pool words: about the first estimate
    assert product_matches(s, s.collect()) == want
    heavy = np.concatenate([key, key + 400])               # twice the keys: the pool overflows
    hval = np.concatenate([val, val])
    s.push(len(heavy), heavy, [hval])
    assert s.attempts() > 1
    got = product_matches(s, s.collect())
    assert len(got) == 2 * len(want)
    for _ in range(2):                                     # the same workload again: the learned size, one attempt
        s.push(len(heavy), heavy, [hval])
        assert s.attempts() == 1
        assert product_matches(s, s.collect()) == got
    for i in range(4):                                     # light batches: the grown pool goes back after the 4th
        s.push(len(light_k), light_k, [light_v])
        assert s.attempts() == 1 and product_matches(s, s.collect()) == light_want
        torch.cuda.synchronize()
        if i < 3:
            assert torch.cuda.mem_get_info()[0] < free0 - (8 << 20)   # still held
    assert torch.cuda.mem_get_info()[0] >= free0 - (64 << 20)          # given back
    # a second session on the same device, with a pool budget the batch cannot fit in (longer keys:
    # their workspace outgrows the first pool estimate, which is linear in the records)
    heavy, hval, _ = synth.c4_stream_np(800, L=19)
    s2 = N.Session(N.CompiledPattern(ir), len(heavy), force_path=N.PATH_GENERAL, lane_nfa=False,
                   max_pool_bytes=12 << 20)              # 3 M words allowed
    s2.push(len(heavy), heavy, [hval])
    out = s2.collect(raise_on_error=False)
    rec, code = s2.batch_errors()
    assert len(code) > 0 and set(int(c) for c in code) == {9}
    failed = set(int(heavy[r]) for r in rec)
    mine = [m for m in product_matches(s2, out) if m[1] not in failed]
    wantk = [m for m in oracle_matches(ir, heavy, [hval], [1], O.MODE_PROCESSOR) if m[1] not in failed]
    assert mine == wantk and len(mine) > 0


def test_segment_count_stays_on_device():
    """After a session's first batch the wave path leaves the batch's segment count on the device
    (NfaArgs.nseg_dev, abi.cpp push_general): no host round trip before the kernel, buffers sized for n
    segments, the pool estimated from the last batch.  Batches with many more keys than the last (the
    pool estimate falls short: the batch re-runs on a larger pool), many fewer, and a single key --
    each against the oracle.  The CSR compaction is enqueued before the host reads the batch's totals
    when the arrays the earlier batches left fit them (the small batches here) and after it otherwise
    (the larger ones)."""
    from kcep import synth
    ir = synth.c4_pattern().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 40000, force_path=N.PATH_GENERAL, lane_nfa=False)
    total = 0
    for nk, L in ((50, 12), (3000, 12), (7, 16), (1, 9), (2000, 8)):
        key, val, _ = synth.c4_stream_np(nk, L=L)
        want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
        s.push(len(key), key, [val])
        got = product_matches(s, s.collect())
        assert got == want, (nk, L)
        total += len(want)
    assert total > 0
