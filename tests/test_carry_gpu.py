"""Per-key state carried across batches (CEP_SESSION_CARRY) against the oracle.

The reference keeps every key's NFA between records in its stores and reloads
it on the next record (CEPProcessor.loadNFA / NFAStore.put,
CEPProcessor.java:111-124, 144-147).  A carry session must therefore produce,
over a stream cut into batches at arbitrary points, exactly the matches of one
uninterrupted run: the oracle processes the concatenated stream in one go and
the device processes it batch by batch (each batch grouped by key), with
record positions reported as stream positions.  The per-key run counter and
queue length (NFATest assertNFA, NFATest.java:836-840) must agree too, and the
state must survive an export/import round trip into a fresh session."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import synth
from golden_util import scenarios, event_arrays
import patterns_lib as PL

pytestmark = pytest.mark.gpu


def oracle_run(ir, key, cols, coltypes, mode, **kw):
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    err = None
    try:
        r.process(O.BatchArrays(key, cols, coltypes, **kw))
    except O.OracleError as e:
        err = (e.code, e.record)
    ms = [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]
    return ms, r, err


def batches_of(key, cuts):
    """Split the stream at `cuts`; every batch is grouped by key (stable), i.e. the
    stream the device sees is the concatenation of the grouped batches."""
    bounds = [0] + sorted(cuts) + [len(key)]
    order = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        order.append(a + np.argsort(key[a:b], kind="stable"))
    return bounds, np.concatenate(order) if order else np.zeros(0, np.int64)


def run_carry(ir, key, cols, bounds, mode=N.MODE_PROCESSOR, max_keys=None, sess=None, lane_nfa=False, **kw):
    cp = N.CompiledPattern(ir) if sess is None else sess.pattern
    if sess is None:
        sess = N.Session(cp, max(1, max(b - a for a, b in zip(bounds[:-1], bounds[1:]))), mode=mode, carry=True,
                         max_keys=max_keys or int(key.max()) + 1, lane_nfa=lane_nfa)
    got = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        if b == a:
            continue
        kw_b = {k: (None if v is None else np.ascontiguousarray(v[a:b])) for k, v in kw.items()}
        sess.push(b - a, np.ascontiguousarray(key[a:b]), [np.ascontiguousarray(c[a:b]) for c in cols], **kw_b)
        out = sess.collect(raise_on_error=False)
        for m in range(len(out["match_record"])):
            x, y = out["ent_off"][m], out["ent_off"][m + 1]
            got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                        [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(x, y)]))
        if out["err"]:
            return got, sess, (int(out["err"]), int(out["err_record"]))
    return got, sess, None


def rand_stream(seed, n_keys, per_key, vmax):
    rng = np.random.default_rng(seed)
    lens = rng.poisson(per_key, n_keys) + 1
    key = np.repeat(np.arange(n_keys, dtype=np.int32), lens)
    rng.shuffle(key)                                    # interleaved arrival, like a topic partition
    val = rng.integers(0, vmax, len(key)).astype(np.int32)
    return key, val


CASES = [
    ("c3_stock", PL.c3_stock, 7, lambda rng, n: (100 + np.cumsum(rng.integers(-5, 6, n))).astype(np.int32)),
    ("c4_any", PL.c4_any, 4, None),
    ("c5_optional", PL.c5_optional, 64, None),
    ("next_one_or_more", PL.next_one_or_more, 4, None),
    ("any_any", PL.any_any, 4, None),
    ("c2_strict", synth.c2_pattern, 4, None),
]


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
@pytest.mark.parametrize("nbatch", [2, 7])
@pytest.mark.parametrize("mode", [N.MODE_PROCESSOR, N.MODE_NFA])
@pytest.mark.parametrize("name,mk,vmax,gen", CASES, ids=[c[0] for c in CASES])
def test_stream_in_batches(name, mk, vmax, gen, mode, nbatch, lane_nfa):
    per_key = 8 if name in ("c4_any", "any_any") else 25
    key, val = rand_stream(len(name) * 7 + nbatch, 150, per_key, vmax)
    if gen is not None:
        val = gen(np.random.default_rng(3), len(key))
    rng = np.random.default_rng(nbatch)
    bounds, order = batches_of(key, list(rng.choice(np.arange(1, len(key)), nbatch - 1, replace=False)))
    key, val = key[order], val[order]
    ir = mk().to_ir(PL.I32)
    omode = O.MODE_PROCESSOR if mode == N.MODE_PROCESSOR else O.MODE_NFA_PER_KEY
    want, r, oerr = oracle_run(ir, key, [val], [1], omode)
    got, sess, gerr = run_carry(ir, key, [val], bounds, mode=mode, lane_nfa=lane_nfa)
    assert oerr is None and gerr is None
    assert len(want) > 0
    assert got == want
    if name == "c3_stock":                              # a runs-path pattern stays on the runs kernels
        assert sess.path == N.PATH_RUNS
    if sess.path in (N.PATH_STENCIL, N.PATH_CHAIN, N.PATH_RUNS):   # carries each key's records, not its queue
        assert name == {N.PATH_STENCIL: "c2_strict", N.PATH_CHAIN: "c5_optional", N.PATH_RUNS: "c3_stock"}[sess.path]
        return
    for k in np.unique(key):                            # NFA.getRuns() and queue length per key
        assert sess.key_state(int(k)) == r.state(int(k)), int(k)


def test_record_at_a_time_integration_fixture():
    """CEPStreamIntegrationTest.java:117-168 driven one record per batch, as the
    reference's processor sees it."""
    fx = [f for f in scenarios() if f["name"] == "integration_multiple_keys"][0]
    a = event_arrays(fx)
    ir = bytes.fromhex(fx["ir"])
    key = a["key"].astype(np.int32)
    kw = {f: a[f] for f in ("topic", "partition", "offset", "ts") if a[f] is not None}
    want, _, _ = oracle_run(ir, key, a["cols"], a["coltypes"], O.MODE_PROCESSOR, **kw)
    got, _, err = run_carry(ir, key, a["cols"], list(range(len(key) + 1)), **kw)
    assert err is None and got == want
    assert len(got) == len(fx["expected"]["sequences"])


def test_export_import_roundtrip():
    """Checkpoint after batch 1 (cep_state_export), restore into a fresh session
    (cep_state_import), continue with batch 2: same matches and state as one session."""
    key, val = rand_stream(5, 200, 30, 4)
    bounds, order = batches_of(key, [len(key) // 2])
    key, val = key[order], val[order]
    ir = PL.next_one_or_more().to_ir(PL.I32)
    whole, s1, _ = run_carry(ir, key, [val], bounds)
    part1, s2, _ = run_carry(ir, key, [val], bounds[:2])
    blob = s2.state_export()
    s3 = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=200)
    s3.state_import(blob)
    assert s3.stream_position() == bounds[1]
    part2, _, _ = run_carry(ir, key, [val], bounds[1:], sess=s3)
    assert part1 + part2 == whole and len(part2) > 0
    for k in range(200):
        assert s3.key_state(k) == s1.key_state(k)
    # a key range exports only those keys
    lo = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=200)
    lo.state_import(s1.state_export(0, 50))
    assert all(lo.key_state(k) is None for k in range(50, 200))
    assert all(lo.key_state(k) == s1.key_state(k) for k in range(50))


def test_high_water_mark_across_batches():
    """CEPProcessor.checkHighWaterMark (:152-160) remembers offsets across batches:
    a record re-delivered in a later batch (same key, value and offset: Kafka
    re-delivery after a failure) is dropped; null records are skipped."""
    rng = np.random.default_rng(11)
    key0, val0 = rand_stream(12, 80, 20, 4)
    n0 = len(key0)
    off0 = np.arange(n0, dtype=np.int64)
    stream = list(range(n0))
    for i in rng.choice(n0, n0 // 6, replace=False):   # re-deliver record i somewhere after it
        j = int(rng.integers(stream.index(i) + 1, len(stream) + 1))
        stream.insert(j, int(i))
    idx = np.array(stream)
    key, val, offset = key0[idx], val0[idx], off0[idx]
    valid = (rng.random(len(idx)) > 0.1).astype(np.uint8)
    bounds, order = batches_of(key, [len(key) // 3, 2 * len(key) // 3])
    key, val, offset, valid = key[order], val[order], offset[order], valid[order]
    ir = PL.any_any().to_ir(PL.I32)
    want, r, _ = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR, offset=offset, valid=valid)
    got, sess, err = run_carry(ir, key, [val], bounds, offset=offset, valid=valid)
    assert err is None and got == want and len(got) > 0


def test_sequence_condition_reads_carried_events():
    """SequenceMatcher averages over the partial sequence (SequenceMatcher.java:21-26):
    with batches of one record every event it averages comes from carried state."""
    fx = [f for f in scenarios() if f["name"] == "nfa_sequence_condition"][0]
    a = event_arrays(fx)
    ir = bytes.fromhex(fx["ir"])
    key = np.zeros(len(a["key"]), np.int32)
    kw = {f: a[f] for f in ("topic", "partition", "offset", "ts") if a[f] is not None}
    want, _, _ = oracle_run(ir, key, a["cols"], a["coltypes"], O.MODE_NFA_PER_KEY, **kw)
    got, _, err = run_carry(ir, key, a["cols"], list(range(len(key) + 1)), mode=N.MODE_NFA, max_keys=1, **kw)
    assert err is None and got == want and len(got) == len(fx["expected"]["sequences"])


def test_key_id_out_of_range_is_rejected():
    ir = PL.any_any().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 10, carry=True, max_keys=4)
    with pytest.raises(N.CepError) as e:
        s.push(2, np.array([1, 9], np.int32), [np.zeros(2, np.int32)])
    assert e.value.code == 11


@pytest.mark.parametrize("mk", [synth.c2_pattern, PL.c5_optional], ids=["stencil", "chain"])
@pytest.mark.parametrize("mem", ["host", "device"])
def test_delivered_batch_with_key_id_out_of_range(mk, mem):
    """CEP_BATCH_DELIVER on a stencil / chain carry session: the delivery kernels run in the same
    stream as the count kernel, before the host sees its error flags, so a match of a key id outside
    [0, max_keys) must not make them read a halo header out of bounds.  The batch fails
    with CEP_E_ARG and the session keeps working."""
    ir = mk().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 64, carry=True, max_keys=4)
    assert s.path in (N.PATH_STENCIL, N.PATH_CHAIN)
    vals = [0, 1, 2] if mk is synth.c2_pattern else [12, 5, 33]
    key = np.array([1, 1, 1, 1 << 20, 1 << 20, 1 << 20], np.int32)
    val = np.array(vals + vals, np.int32)
    if mem == "device":
        import torch
        dk, dv = torch.from_numpy(key).cuda(), torch.from_numpy(val).cuda()
        torch.cuda.synchronize()
        push = lambda: s.push(len(key), dk.data_ptr(), [dv.data_ptr()], mem=N.MEM_DEVICE,
                              flags=N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER)
    else:
        push = lambda: s.push(len(key), key, [val], flags=N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER)
    with pytest.raises(N.CepError) as e:
        push()
        s.collect()
    assert e.value.code == 11
    s.push(3, key[:3], [val[:3]], flags=N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER)   # the session still works
    assert len(s.collect()["match_record"]) == 1


def test_interleaved_carry_batch_is_rejected():
    """A carry batch must hold each key in one contiguous segment (kcep.h batch contract): a key
    in two segments would load its carried state twice and lose one segment's update, so the
    push fails with CEP_E_ARG before the NFA runs, and the carried state is untouched."""
    ir = PL.any_any().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 10, carry=True, max_keys=4)
    s.push(3, np.array([0, 0, 1], np.int32), [np.array([0, 1, 2], np.int32)])
    s.collect()
    before = [s.key_state(k) for k in range(4)]
    with pytest.raises(N.CepError) as e:
        s.push(3, np.array([0, 1, 0], np.int32), [np.array([1, 2, 3], np.int32)])
    assert e.value.code == 11
    assert [s.key_state(k) for k in range(4)] == before
    s.push(2, np.array([1, 1], np.int32), [np.array([1, 2], np.int32)])   # the session still works
    s.collect()


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_stencil_carry_record_at_a_time(k):
    """Strict k-stage patterns stay on the stencil path with carried state: each key's last k-1 records
    (the halo) cross batch boundaries.  Batches of 1, 2 and 5 records: most matches take their first
    stages from the halo."""
    rng = np.random.default_rng(k)
    key = rng.integers(0, 7, 400).astype(np.int32)
    val = rng.integers(0, 2, 400).astype(np.int32)
    q = PL.QueryBuilder().select("s0").where(PL.Event.value() == 0)
    for i in range(1, k):
        q = q.then().select(f"s{i}").where(PL.Event.value() == (i % 2))
    ir = q.build().to_ir(PL.I32)
    want, _, oerr = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    assert oerr is None and len(want) > 0
    for step in (1, 2, 5):
        bounds, order = batches_of(key, list(range(step, len(key), step)))
        got, sess, err = run_carry(ir, key[order], [val[order]], bounds, max_keys=7)
        assert sess.path == N.PATH_STENCIL and err is None
        # the device saw the grouped batches: map its stream positions back to arrival order
        got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
        assert sorted(got) == sorted(want)


def test_stencil_carry_export_import():
    """A stencil carry session's halos (cep_state_export "KCSH") restored into a fresh session: the
    rest of the stream continues as in one session."""
    key, val = rand_stream(21, 300, 20, 4)
    bounds, order = batches_of(key, [len(key) // 3, 2 * len(key) // 3])
    key, val = key[order], val[order]
    ir = synth.c2_pattern().to_ir(PL.I32)
    whole, s1, _ = run_carry(ir, key, [val], bounds)
    part1, s2, _ = run_carry(ir, key, [val], bounds[:2])
    assert s1.path == N.PATH_STENCIL
    blob = s2.state_export()
    assert blob[:4] == b"KCSH"
    s3 = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=300)
    s3.state_import(blob)
    assert s3.stream_position() == bounds[1]
    part2, _, _ = run_carry(ir, key, [val], bounds[1:], sess=s3)
    assert part1 + part2 == whole and len(part2) > 0


def test_stencil_carry_rejects_unclean_batches():
    ir = synth.c2_pattern().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 10, carry=True, max_keys=4)
    assert s.path == N.PATH_STENCIL
    with pytest.raises(N.CepError) as e:
        s.push(2, np.array([1, 1], np.int32), [np.zeros(2, np.int32)], valid=np.ones(2, np.uint8))
    assert e.value.code == 12
    with pytest.raises(N.CepError) as e:                 # interleaved keys: found at collect
        s.push(3, np.array([1, 2, 1], np.int32), [np.zeros(3, np.int32)])
        s.collect()
    assert e.value.code == 11


CHAIN_PATTERNS = {
    # A B? C where a record can end two runs at once (0 1 2: A B C, and A(1) skip-B C)
    "abc3": lambda v: (PL.QueryBuilder().select("a").where((v == 0) | (v == 1)).then()
                       .select("b").optional().where(v == 1).then().select("c").where(v == 2).build()),
    # A B? C? D: two optional stages, runs reaching back K-1 = 3 records
    "abcd4": lambda v: (PL.QueryBuilder().select("a").where(v <= 1).then()
                        .select("b").optional().where(v == 1).then()
                        .select("c").optional().where((v == 2) | (v == 1)).then()
                        .select("d").where(v >= 2).build()),
}


@pytest.mark.parametrize("name", list(CHAIN_PATTERNS))
def test_chain_carry_record_at_a_time(name):
    """Chain patterns (strict with optional() stages) keep their carried state on the chain path:
    runs that started in a key's halo are replayed at the key's first records of the next batch.
    Batches of 1, 2, 3 and 7 records against one oracle run of the whole stream."""
    rng = np.random.default_rng(len(name))
    key = rng.integers(0, 5, 600).astype(np.int32)
    val = rng.integers(0, 4, 600).astype(np.int32)
    ir = CHAIN_PATTERNS[name](PL.Event.value()).to_ir(PL.I32)
    want, _, oerr = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    assert oerr is None and len(want) > 0
    for step in (1, 2, 3, 7):
        bounds, order = batches_of(key, list(range(step, len(key), step)))
        got, sess, err = run_carry(ir, key[order], [val[order]], bounds, max_keys=5)
        assert sess.path == N.PATH_CHAIN and err is None
        got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
        # per key the matches keep the reference's order (record, then oldest start first)
        assert sorted(got) == sorted(want)
        for k in range(5):
            assert [m for m in got if m[1] == k] == [m for m in want if m[1] == k]


def test_chain_carry_c5_random_cuts_and_export():
    """C5's pattern streamed in random cuts (arrival order kept by grouping each batch), then a
    checkpoint (KCSH) restored into a fresh session mid-stream."""
    key, val = rand_stream(33, 400, 30, 64)
    ir = synth.c5_pattern().to_ir(PL.I32)
    rng = np.random.default_rng(4)
    bounds, order = batches_of(key, list(rng.choice(np.arange(1, len(key)), 9, replace=False)))
    key, val = key[order], val[order]
    want, _, _ = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    whole, s1, err = run_carry(ir, key, [val], bounds)
    assert s1.path == N.PATH_CHAIN and err is None and whole == want and len(want) > 0
    half = len(bounds) // 2
    part1, s2, _ = run_carry(ir, key, [val], bounds[:half + 1])
    blob = s2.state_export()
    assert blob[:4] == b"KCSH"
    s3 = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=400)
    s3.state_import(blob)
    part2, _, _ = run_carry(ir, key, [val], bounds[half:], sess=s3)
    assert part1 + part2 == whole


# ---- the runs path's carried tails (runs.hip): each key's records from its oldest open run on ----

def c3_stream(seed, n_keys, per_key):
    rng = np.random.default_rng(seed)
    key = np.repeat(np.arange(n_keys, dtype=np.int32), rng.poisson(per_key, n_keys) + 1)
    rng.shuffle(key)
    val = (100 + np.cumsum(rng.integers(-5, 6, len(key)))).astype(np.int32)
    return key, val


@pytest.mark.parametrize("cuts", [1, 2, 5, 64])
def test_runs_carry_cut_anywhere(cuts):
    """C3's pattern (stock oneOrMore + sum/count folds) on the runs path of a carry session, the
    stream cut into batches of `cuts` records (1: record at a time): open runs -- with their fold
    registers -- continue across every cut, as the reference's NFAStore/AggregatesStore keep them
    (CEPProcessor.java:111-124, 144-147; AggregatesStoreImpl.java:55-75)."""
    key, val = c3_stream(cuts, 60 if cuts < 5 else 200, 12 if cuts < 5 else 30)
    bounds, order = batches_of(key, list(range(cuts, len(key), cuts)))
    key, val = key[order], val[order]
    ir = PL.c3_stock().to_ir(PL.I32)
    want, _, oerr = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    got, sess, gerr = run_carry(ir, key, [val], bounds)
    assert sess.path == N.PATH_RUNS
    assert oerr is None and gerr is None
    assert len(want) > 0 and got == want


def test_runs_carry_long_open_run_and_export_import():
    """A oneOrMore run that stays open over many batches (rising prices keep avg < v), then a
    mid-stream checkpoint (cep_state_export "KCSR") restored into a fresh session: the rest of the
    stream matches as one uninterrupted run, and cep_state_positions lists the carried records."""
    from kcep import native as NN
    n_keys = 8
    rng = np.random.default_rng(3)
    key = np.tile(np.arange(n_keys, dtype=np.int32), 150)
    val = (100 + np.arange(len(key)) // n_keys + rng.integers(0, 2, len(key))).astype(np.int32)  # slow rise
    val[len(val) * 3 // 4:] -= 40                                            # then a drop closes the runs
    ir = PL.c3_stock().to_ir(PL.I32)
    want, _, _ = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    bounds = list(range(0, len(key), 16)) + [len(key)]
    order = np.concatenate([a + np.argsort(key[a:b], kind="stable") for a, b in zip(bounds[:-1], bounds[1:])])
    key, val = key[order], val[order]
    want, _, _ = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    half = len(bounds) // 2
    got, s1, _ = run_carry(ir, key, [val], bounds[:half + 1], max_keys=n_keys)
    blob = s1.state_export()
    assert blob[:4] == b"KCSR"
    pos = NN.state_positions(blob)
    assert len(pos) > 0 and pos.max() < bounds[half]
    s2 = N.Session(N.CompiledPattern(ir), 16, carry=True, max_keys=n_keys)
    s2.state_import(blob)
    assert s2.stream_position() == bounds[half]
    rest = [b - bounds[half] for b in bounds[half:]]
    got2, _, _ = run_carry(ir, key[bounds[half]:], [val[bounds[half]:]], rest, sess=s2)
    assert len(want) > 0 and got + got2 == want


@pytest.mark.parametrize("bad", ["key_out_of_range", "key_in_two_segments"])
def test_runs_carry_rejected_batch_leaves_tails(bad):
    """A runs-path carry batch is launched before the host has read its key checks (the extended
    batch's size stays on the device: one synchronisation per batch).  A batch with a key id outside
    [0, max_keys) or a key in two segments still fails with CEP_E_ARG, its tail kernels leave the
    carried tails and the key table as they were, and the stream continues exactly as the oracle's
    without that batch (open runs carried across it)."""
    ir = PL.c3_stock().to_ir(PL.I32)
    key, val = c3_stream(3, 40, 12)
    bounds, order = batches_of(key, list(range(20, len(key), 20)))
    key, val = key[order], val[order]
    want, _, oerr = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), len(key) + 8, carry=True, max_keys=64)
    assert s.path == N.PATH_RUNS
    got = []
    for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        if i == len(bounds) // 2:
            if bad == "key_out_of_range":
                bk, bv = np.array([1, 1, 1 << 20, 1 << 20], np.int32), np.array([5, 6, 7, 8], np.int32)
            else:
                bk, bv = np.array([1, 2, 1], np.int32), np.array([5, 6, 7], np.int32)
            with pytest.raises(N.CepError) as e:
                s.push(len(bk), bk, [bv], flags=N.BATCH_OFFSETS_MONOTONE)
            assert e.value.code == 11
        s.push(b - a, key[a:b], [val[a:b]], flags=N.BATCH_OFFSETS_MONOTONE)
        out = s.collect()
        got += [(int(out["match_record"][m]), int(out["match_key"][m])) for m in range(len(out["match_record"]))]
    assert oerr is None and len(want) > 0
    assert got == [(m[0], m[1]) for m in want]


def test_runs_carry_duplicate_key_with_a_long_tail_is_bounded():
    """a runs carry batch is launched on a bound of its extended size (the batch plus
    every tail record the pool holds) before its key check is read.  A batch holding key 0 in two
    segments gives key 0's tail to both, which can exceed that bound when key 0's tail is more than half
    of the live tails -- here right after the first batch (no garbage in the pool yet: the bound is the
    live tails exactly) with key 0 holding almost all of them.  The writes past the bound are dropped on
    the device, the batch fails with CEP_E_ARG, and the stream then continues as the oracle's without it."""
    ir = PL.c3_stock().to_ir(PL.I32)
    n0 = 600
    key = np.concatenate([np.zeros(n0, np.int32), np.ones(4, np.int32)])
    # key 0: a constant price keeps every run open (avg >= v, never avg < v): its tail is its whole segment
    val = np.concatenate([np.full(n0, 100), [100, 99, 98, 97]]).astype(np.int32)
    tail_k = np.concatenate([np.zeros(3, np.int32), np.ones(2, np.int32)])
    tail_v = np.array([200, 90, 80, 200, 50], np.int32)                                 # closes / continues the runs
    want, _, oerr = oracle_run(ir, np.concatenate([key, tail_k]), [np.concatenate([val, tail_v])], [1],
                               O.MODE_PROCESSOR)
    s = N.Session(N.CompiledPattern(ir), 2 * n0, carry=True, max_keys=4)
    assert s.path == N.PATH_RUNS
    s.push(len(key), key, [val], flags=N.BATCH_OFFSETS_MONOTONE)
    got = s.collect()
    got = [(int(got["match_record"][m]), int(got["match_key"][m])) for m in range(len(got["match_record"]))]
    blob = s.state_export()
    assert len(NN_state_positions(blob)) >= n0 - 1          # key 0 carries (nearly) its whole segment
    for _ in range(3):
        with pytest.raises(N.CepError) as e:
            s.push(5, np.array([0, 0, 1, 0, 0], np.int32), [np.array([5, 6, 7, 8, 9], np.int32)],
                   flags=N.BATCH_OFFSETS_MONOTONE)
        assert e.value.code == 11
    s.push(len(tail_k), tail_k, [tail_v], flags=N.BATCH_OFFSETS_MONOTONE)
    out = s.collect()
    got += [(int(out["match_record"][m]), int(out["match_key"][m])) for m in range(len(out["match_record"]))]
    assert oerr is None and len(want) > 0
    assert got == [(m[0], m[1]) for m in want]


def NN_state_positions(blob):
    from kcep import native as NN
    return NN.state_positions(blob)


def test_runs_carry_rejects_unclean_batches():
    """Like the stencil carry: null records or unflagged offsets cannot be taken by the runs kernels
    (the host applies CEPProcessor's filters first)."""
    ir = PL.c3_stock().to_ir(PL.I32)
    s = N.Session(N.CompiledPattern(ir), 8, carry=True, max_keys=4)
    assert s.path == N.PATH_RUNS
    key = np.array([0, 0, 1, 1], np.int32)
    val = np.array([100, 101, 102, 103], np.int32)
    with pytest.raises(N.CepError) as ei:
        s.push(4, key, [val], offset=np.arange(4, dtype=np.int64))
    assert ei.value.code == 12
    s.push(4, key, [val], offset=np.arange(4, dtype=np.int64), flags=N.BATCH_OFFSETS_MONOTONE)
    s.collect()


def _strict_pattern(k):
    q = PL.QueryBuilder().select("s0").where(PL.Event.value() == 0)
    for i in range(1, k):
        q = q.then().select(f"s{i}").where(PL.Event.value() == (i % 2))
    return q.build().to_ir(PL.I32)


@pytest.mark.parametrize("k", [2, 3, 5, 7])
def test_stencil_carry_large_batches(k):
    """Carry batches of many tiles (the plain kernel's carry variant): segments of every length from
    1 record up cross lane, wave (256-record) and tile (4096-record) boundaries, keys continue across
    3 batch cuts; against one oracle run of the whole stream."""
    rng = np.random.default_rng(100 + k)
    n_keys = 600
    lens = np.concatenate([rng.integers(1, 8, 200), rng.poisson(400, n_keys - 200) + 1])
    key = np.repeat(rng.permutation(n_keys).astype(np.int32), lens)
    rng.shuffle(key)
    val = rng.integers(0, 2, len(key)).astype(np.int32)
    ir = _strict_pattern(k)
    want, _, oerr = oracle_run(ir, key, [val], [1], O.MODE_PROCESSOR)
    assert oerr is None and len(want) > 1000
    cuts = sorted(rng.choice(np.arange(1, len(key)), 3, replace=False).tolist())
    bounds, order = batches_of(key, cuts)
    got, sess, err = run_carry(ir, key[order], [val[order]], bounds, max_keys=n_keys)
    assert sess.path == N.PATH_STENCIL and err is None
    got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
    assert sorted(got) == sorted(want)


def test_stencil_carry_large_batch_key_in_two_segments():
    """A key in two segments of one large batch (in different workgroups' tiles) is the
    interleaved-batch error (CEP_E_ARG at collect), as for a small batch."""
    ir = synth.c2_pattern().to_ir(PL.I32)
    key = np.repeat(np.arange(300, dtype=np.int32), 100)
    key[20000:20100] = 7                                 # key 7 again, ~13k records after its segment
    s = N.Session(N.CompiledPattern(ir), len(key), carry=True, max_keys=300)
    assert s.path == N.PATH_STENCIL
    with pytest.raises(N.CepError) as e:
        s.push(len(key), key, [np.zeros(len(key), np.int32)])
        s.collect()
    assert e.value.code == 11


@pytest.mark.parametrize("k", [2, 3])
def test_stencil_carry_partial_last_super_tile(k):
    """A batch of 8193 tiles runs 4 tiles per workgroup, the last workgroup one tile: its boundary
    matches' aux bytes lie past its own tile's slot ints (the slot buffer is padded for them).  Keys
    of the first batch continue in the second batch's last tile, behind 33.5 M filler records that
    match nothing; the matches equal the oracle's over the first batch plus that tail."""
    rng = np.random.default_rng(7 + k)
    nk = 40
    b1_key = np.repeat(np.arange(nk, dtype=np.int32), 3)
    b1_val = rng.integers(0, 2, len(b1_key)).astype(np.int32)
    n2 = 8193 * 4096
    tail = 2048
    t_key = np.sort(rng.integers(0, nk, tail)).astype(np.int32)
    t_val = rng.integers(0, 2, tail).astype(np.int32)
    f_key = (nk + np.arange(n2 - tail) // 1000).astype(np.int32)     # filler keys, segments of 1000
    key2 = np.concatenate([f_key, t_key])
    val2 = np.concatenate([np.full(n2 - tail, 3, np.int32), t_val])
    ir = _strict_pattern(k)
    # the oracle over the first batch and the tail (the filler shares no key with them)
    o_key = np.concatenate([b1_key, t_key])
    o_val = np.concatenate([b1_val, t_val])
    want, _, oerr = oracle_run(ir, o_key, [o_val], [1], O.MODE_PROCESSOR)
    assert oerr is None and len(want) > 20
    shift = n2 - tail                                  # oracle position p >= len(b1) -> stream position p + shift

    def pos(p):
        return p if p < len(b1_key) else p + shift
    want = sorted((pos(m[0]), m[1], [(nm, pos(r)) for nm, r in m[2]]) for m in want)
    s = N.Session(N.CompiledPattern(ir), n2, carry=True, max_keys=int(key2.max()) + 1)
    got, s, err = run_carry(ir, np.concatenate([b1_key, key2]), [np.concatenate([b1_val, val2])],
                            [0, len(b1_key), len(b1_key) + n2], sess=s)
    assert s.path == N.PATH_STENCIL and err is None
    assert sorted(got) == want
    assert any(r < len(b1_key) for m in got for _, r in m[2])   # matches that start in the halo


@pytest.mark.parametrize("t", ["i32_topic", "i64", "f64"])
def test_stencil_carry_topic_and_wide_columns(t):
    """The plain carry kernel's topic and 64-bit value instantiations: multi-tile batches with keys
    continuing across 3 cuts, against one oracle run of the whole stream."""
    from kcep import Schema, QueryBuilder, Event, Selected
    rng = np.random.default_rng(31)
    n_keys = 300
    key = np.repeat(rng.permutation(n_keys).astype(np.int32), rng.poisson(150, n_keys) + 1)
    rng.shuffle(key)
    n = len(key)
    kw, ty = {}, 1
    if t == "i32_topic":
        val = rng.integers(0, 3, n).astype(np.int32)
        kw["topic"] = rng.integers(0, 2, n).astype(np.int32)
        sch = Schema([("value", "i32")], topics=["t0", "t1"])
        q = (QueryBuilder().select("a", Selected.withStrictContiguity().withTopic("t1")).where(Event.value() == 0)
             .then().select("b").where(Event.value() != 0).then()
             .select("c", Selected.withStrictContiguity().withTopic("t0")).where(Event.value() == 2).build())
    else:
        raw = rng.integers(-3, 4, n)
        c = 1_000_000_007 if t == "i64" else 0.5
        val = (raw * c).astype(np.int64) if t == "i64" else raw.astype(np.float64) * 0.5
        ty = 2 if t == "i64" else 3
        sch = Schema([("value", t)])
        q = (QueryBuilder().select("lo").where(Event.value() < 0).then()
             .select("hi").where(Event.value() > c).build())
    ir = q.to_ir(sch)
    want, _, oerr = oracle_run(ir, key, [val], [ty], O.MODE_PROCESSOR, **kw)
    assert oerr is None and len(want) > 100
    cuts = sorted(rng.choice(np.arange(1, n), 3, replace=False).tolist())
    bounds, order = batches_of(key, cuts)
    got, sess, err = run_carry(ir, key[order], [val[order]], bounds, max_keys=n_keys,
                               **{f: v[order] for f, v in kw.items()})
    assert sess.path == N.PATH_STENCIL and err is None
    got = [(int(order[m[0]]), m[1], [(nm, int(order[r])) for nm, r in m[2]]) for m in got]
    assert sorted(got) == sorted(want)
