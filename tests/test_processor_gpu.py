"""GpuCEPProcessor (kcep/processor.py) end to end on the device.

The processor is the batching equivalent of the reference's CEPProcessor
(CEPProcessor.java:111-160): records go in one at a time with their context
(topic, partition, offset, timestamp), values are decoded into SoA columns, and
forwarded (key, Sequence) pairs come out.  Its forwarded stream must equal the
reference's record for record, whatever the batch size:

* the reference's own processor-mode fixtures (CEPStockDemoTest with values as
  StockEventSerde JSON bytes, CEPStreamIntegrationTest multiple keys),
* random interleaved streams with nulls and re-delivered offsets against the
  oracle run over the same arrival-order stream,
* a checkpoint/restore into a fresh processor mid-stream,
* the reference's exception, raised after forwarding what came before it.
"""
import numpy as np
import pytest

import oracle as O
from kcep import Schema
from kcep import native as N
from kcep.ingest import StockEvent, StockEventSerde, ColumnDecoder, stock_columns, scalar_column, STOCK_SCHEMA
from kcep.processor import GpuCEPProcessor, ProcessorFailed
from kcep.sequence import Event as Ev, sequence_from_traversal
from golden_util import scenarios
import patterns_lib as PL
from kcep import synth

pytestmark = pytest.mark.gpu


def seq_view(seq):
    return [(s.getStage(), [e.offset for e in s.getEvents()]) for s in seq.matched()]


def run_proc(proc, records, flush_every=None):
    got = []
    proc.init(lambda k, s: got.append((k, seq_view(s))))
    for i, r in enumerate(records):
        proc.process(*r)
        if flush_every and (i + 1) % flush_every == 0:
            proc.punctuate(0)
    proc.close()
    return got


def fixture(name):
    return [f for f in scenarios() if f["name"] == name][0]


@pytest.mark.parametrize("batch", [1, 3, 8, 1000])
def test_stock_demo_from_json_bytes(batch):
    """CEPStockDemoTest.java:97-138: quotes serialized by StockEventSerde, decoded by the
    processor's ingest path, matched on the device, forwarded as Sequences."""
    fx = fixture("stock_demo")
    ev = fx["events"]
    recs = []
    for i in range(len(ev["key"])):
        data = StockEventSerde.serialize("stock-events", StockEvent("ALXN", ev["cols"][0][i], ev["cols"][1][i]))
        val = StockEventSerde.deserialize("stock-events", data)
        recs.append(("ALXN", val, "stock-events", 0, ev["offset"][i], ev["ts"][i]))
    proc = GpuCEPProcessor("Stocks", bytes.fromhex(fx["ir"]), STOCK_SCHEMA, stock_columns(), batch_size=batch)
    got = run_proc(proc, recs)
    want = [("ALXN", [(g["stage"], g["events"]) for g in s]) for s in fx["expected"]["sequences"]]
    assert got == want


@pytest.mark.parametrize("batch", [1, 4, 100])
def test_integration_multiple_keys(batch):
    """CEPStreamIntegrationTest.java:117-168 through the processor."""
    fx = fixture("integration_multiple_keys")
    ev = fx["events"]
    sch = Schema([("value", "i32")], topics=list(fx["topics"]))
    ir = bytes.fromhex(fx["ir"])
    recs = [(f"K{ev['key'][i]}", ev["cols"][0][i], "input_topic_1", 0, ev["offset"][i], ev["ts"][i])
            for i in range(len(ev["key"]))]
    proc = GpuCEPProcessor("Integration", ir, sch, scalar_column(sch), batch_size=batch)
    got = run_proc(proc, recs)
    want = [(f"K{k}", [(g["stage"], g["events"]) for g in s])
            for k, s in zip(fx["expected"]["match_keys"], fx["expected"]["sequences"])]
    assert got == want


def random_records(seed, n_keys, n, vmax, null_frac=0.05, redeliver_frac=0.05):
    """Interleaved keys, offsets increasing per partition, some nulls, some re-deliveries."""
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        k = int(rng.integers(0, n_keys))
        v = int(rng.integers(0, vmax))
        recs.append([f"user-{k}", v, "events", 0, i, 1000 + i])
    for _ in range(int(n * redeliver_frac)):            # the same record delivered again later
        i = int(rng.integers(0, n))
        j = int(rng.integers(i + 1, len(recs) + 1))
        recs.insert(j, list(recs[i]))
    for i in rng.choice(len(recs), int(len(recs) * null_frac), replace=False):
        if rng.random() < 0.5:
            recs[i][0] = None
        else:
            recs[i][1] = None
    return [tuple(r) for r in recs]


def oracle_forward(pattern, sch, recs):
    """The oracle over the arrival-order stream (processor mode), as (key, sequence view)."""
    keys = {}
    kid, val, valid, off, ts = [], [], [], [], []
    for k, v, _t, _p, o, t in recs:
        kid.append(keys.setdefault(k, len(keys)) if k is not None else 0)
        val.append(0 if v is None else v)
        valid.append(0 if (k is None or v is None) else 1)
        off.append(o)
        ts.append(t)
    p = O.OraclePattern(pattern.to_ir(sch))
    r = O.OracleRun(p, O.MODE_PROCESSOR)
    r.process(O.BatchArrays(np.asarray(kid, np.int32), [np.asarray(val, np.int32)], [1],
                            valid=np.asarray(valid, np.uint8), offset=np.asarray(off, np.int64),
                            ts=np.asarray(ts, np.int64)))

    def event_of(i):
        k, v, t, pa, o, ts_ = recs[i]
        return Ev(k, v, ts_, t, pa, o)
    out = []
    for m in r.matches(with_groups=False):
        seq = sequence_from_traversal(m.traversal, p.names, event_of)
        out.append((recs[m.record][0], seq_view(seq)))
    return out


@pytest.mark.parametrize("name,mk,vmax", [("any_any", PL.any_any, 4), ("next_one_or_more", PL.next_one_or_more, 4),
                                          ("c3_stock", PL.c3_stock, 7), ("c2_strict", synth.c2_pattern, 4)])
@pytest.mark.parametrize("batch", [7, 256])
def test_random_streams_vs_oracle(name, mk, vmax, batch):
    recs = random_records(sum(map(ord, name)) * 31 + batch, 40, 1500, vmax)
    if name == "c3_stock":                              # a price walk, so the averages move
        walk = 100 + np.cumsum(np.random.default_rng(3).integers(-5, 6, len(recs)))
        recs = [(k, None if v is None else int(walk[i]), t, p, o, ts) for i, (k, v, t, p, o, ts) in enumerate(recs)]
    sch = Schema([("value", "i32")])
    want = oracle_forward(mk(), sch, recs)
    proc = GpuCEPProcessor(name, mk(), sch, scalar_column(sch), batch_size=batch)
    got = run_proc(proc, recs)
    assert len(want) > 0
    assert got == want
    if name == "c2_strict":                             # strict fixed-length: the stencil kernel, carried
        assert proc.compiled.info.stencil_ok


@pytest.mark.parametrize("name,mk,vmax", [("any_any", PL.any_any, 4), ("c3_stock", PL.c3_stock, 7),
                                          ("c2_strict", synth.c2_pattern, 4), ("c5", synth.c5_pattern, 64)])
def test_more_distinct_keys_than_max_keys(name, mk, vmax):
    """VERDICT r2 #8 / NFAStoreImpl.java:34-85 (unbounded): 500 distinct keys through a processor
    whose session holds 48 key ids.  Cold keys are spilled to the host (cep_state_evict) and come
    back under other ids (cep_state_import_keys) with their runs and marks; the forwarded stream
    equals the oracle's, and a checkpoint taken mid-stream (spilled keys included) restores."""
    recs = random_records(77 + len(name), 500, 4000, vmax)
    if name == "c3_stock":
        walk = 100 + np.cumsum(np.random.default_rng(4).integers(-5, 6, len(recs)))
        recs = [(k, None if v is None else int(walk[i]), t, p, o, ts) for i, (k, v, t, p, o, ts) in enumerate(recs)]
    sch = Schema([("value", "i32")])
    want = oracle_forward(mk(), sch, recs)
    proc = GpuCEPProcessor(name, mk(), sch, scalar_column(sch), batch_size=40, max_keys=48, prune_at=300)
    got = run_proc(proc, recs)
    assert len(want) > 0 and got == want
    assert proc._spilled or proc._next_id == 48
    # checkpoint / restore with spilled keys
    half = len(recs) // 2
    p1 = GpuCEPProcessor(name, mk(), sch, scalar_column(sch), batch_size=40, max_keys=48)
    g1 = []
    p1.init(lambda k, s: g1.append((k, seq_view(s))))
    for r in recs[:half]:
        p1.process(*r)
    snap = p1.checkpoint()
    assert snap["spilled"]
    p1.close()
    s2 = Schema([("value", "i32")])
    p2 = GpuCEPProcessor(name, mk(), s2, scalar_column(s2), batch_size=40, max_keys=48)
    p2.init(lambda k, s: g1.append((k, seq_view(s))))
    p2.restore(snap)
    for r in recs[half:]:
        p2.process(*r)
    p2.close()
    assert g1 == want


def test_capacity_key_is_rerun_with_the_cap_lifted():
    """a key over cep_opts.max_key_words is handed back with CEP_E_RUN_CAPACITY and
    its state as of the batch start; the processor re-pushes exactly that key's records with the
    cap lifted, so nothing is lost and the forwarded stream is the oracle's."""
    rng = np.random.default_rng(12)
    recs = []
    for i in range(3000):
        k = 3 if rng.random() < 0.1 else int(rng.integers(0, 60))
        recs.append((f"user-{k}", int(rng.integers(0, 4)), "events", 0, i, i))
    sch = Schema([("value", "i32")])
    want = oracle_forward(PL.any_any(), sch, recs)
    proc = GpuCEPProcessor("cap", PL.any_any(), sch, scalar_column(sch), batch_size=1000, max_key_words=1 << 15)
    got = run_proc(proc, recs)
    assert proc.capacity_reruns > 0
    assert got == want


def test_checkpoint_restore_mid_stream():
    """Checkpoint (cep_state_export + key table + carried records) half way, restore into a
    fresh processor, continue: the same forwarded stream as one uninterrupted processor."""
    recs = random_records(77, 30, 1200, 4)
    sch = Schema([("value", "i32")])
    whole = run_proc(GpuCEPProcessor("q", PL.next_one_or_more(), sch, scalar_column(sch), batch_size=64), recs)

    got = []
    fwd = lambda k, s: got.append((k, seq_view(s)))   # noqa: E731
    p1 = GpuCEPProcessor("q", PL.next_one_or_more(), sch, scalar_column(sch), batch_size=64)
    p1.init(fwd)
    half = len(recs) // 2
    for r in recs[:half]:
        p1.process(*r)
    snap = p1.checkpoint()
    p1.close()
    p2 = GpuCEPProcessor("q", PL.next_one_or_more(), sch, scalar_column(sch), batch_size=64)
    p2.init(fwd)
    p2.restore(snap)
    for r in recs[half:]:
        p2.process(*r)
    p2.close()
    assert got == whole and len(whole) > 0


def test_checkpoint_restore_fresh_schema_two_topics():
    """High-water marks are carried per interned topic id (NFAStates.java:37): a restore into a
    processor with a freshly built Schema that meets the topics in the other order must keep
    the snapshot's ids, or re-delivered records are judged against the wrong topic's mark."""
    rng = np.random.default_rng(5)
    recs, off = [], {"ta": 1000, "tb": 0}
    for i in range(1600):
        t = "ta" if i < 400 else ("tb" if i < 900 or rng.random() < 0.5 else "ta")
        recs.append((f"user-{int(rng.integers(0, 20))}", int(rng.integers(0, 4)), t, 0, off[t], i))
        off[t] += 1
    half = 1000                                         # the second half starts with topic tb
    recs = recs[:half] + [recs[i] for i in rng.choice(half, 60)] + recs[half:]   # re-deliveries
    whole = run_proc(GpuCEPProcessor("q", PL.any_any(), Schema([("value", "i32")]),
                                     scalar_column(Schema([("value", "i32")])), batch_size=64), recs)
    got = []
    fwd = lambda k, s: got.append((k, seq_view(s)))   # noqa: E731
    s1 = Schema([("value", "i32")])
    p1 = GpuCEPProcessor("q", PL.any_any(), s1, scalar_column(s1), batch_size=64)
    p1.init(fwd)
    for r in recs[:half]:
        p1.process(*r)
    snap = p1.checkpoint()
    p1.close()
    s2 = Schema([("value", "i32")])                     # fresh: no topic seen yet
    p2 = GpuCEPProcessor("q", PL.any_any(), s2, scalar_column(s2), batch_size=64)
    p2.init(fwd)
    p2.restore(snap)
    assert s2.topics == {"ta": 0, "tb": 1}
    for r in recs[half:]:
        p2.process(*r)
    p2.close()
    assert got == whole and len(whole) > 0
    s3 = Schema([("value", "i32")], topics=["tb"])      # an id already taken by another topic
    p3 = GpuCEPProcessor("q", PL.any_any(), s3, scalar_column(s3), batch_size=64)
    p3.init(fwd)
    with pytest.raises(ProcessorFailed):
        p3.restore(snap)
    p3.close()


def test_reference_exception_surfaces():
    """test_stock_demo_minimal_npe's input through the processor: the matches before the
    failing record are forwarded, then the reference's NullPointerException is raised and
    the processor stays failed."""
    quotes = [(100, 1001), (102, 1001), (102, 700), (100, 500)]
    recs = [("S", StockEvent("S", p, v), "stock-events", 0, i, i) for i, (p, v) in enumerate(quotes)]
    got = []
    proc = GpuCEPProcessor("Stocks", PL.stock_demo(), STOCK_SCHEMA, stock_columns(), batch_size=16)
    proc.init(lambda k, s: got.append((k, seq_view(s))))
    for r in recs:
        proc.process(*r)
    with pytest.raises(N.CepError) as ei:
        proc.flush()
    assert ei.value.code == 4 and ei.value.record == 3
    want = oracle_forward_stock(quotes)
    assert got == want
    with pytest.raises(ProcessorFailed):
        proc.process(*recs[0])


def oracle_forward_stock(quotes):
    p = O.OraclePattern(PL.stock_demo().to_ir(STOCK_SCHEMA))
    r = O.OracleRun(p, O.MODE_PROCESSOR)
    n = len(quotes)
    with pytest.raises(O.OracleError) as ei:
        r.process(O.BatchArrays(np.zeros(n, np.int32), [np.array([q[0] for q in quotes], np.int64),
                                                         np.array([q[1] for q in quotes], np.int64)], [2, 2]))
    return [("S", seq_view(sequence_from_traversal(m.traversal, p.names,
                                                   lambda i: Ev("S", None, i, "stock-events", 0, i))))
            for m in r.matches(with_groups=False) if m.record < ei.value.record]   # forward() runs after
                                                                                 # matchPattern returns (:142-148)


@pytest.mark.parametrize("seed", [11, 17, 28])
def test_stock_demo_random_keys_fail_where_the_reference_fails(seed):
    """The example pattern on random interleaved quotes of 200 keys throws inside the
    reference (test_stock_demo_random); several keys fail within one batch.  The processor
    must forward exactly what the reference forwarded before its first exception in
    arrival order, and raise that exception at that record."""
    rng = np.random.default_rng(seed)
    n = 5000
    kid = rng.integers(0, 200, n).astype(np.int32)
    price = (120 + rng.integers(-6, 7, n)).astype(np.int64)
    vol = rng.integers(600, 1200, n).astype(np.int64)
    p = O.OraclePattern(PL.stock_demo().to_ir(STOCK_SCHEMA))
    r = O.OracleRun(p, O.MODE_PROCESSOR)
    with pytest.raises(O.OracleError) as oe:
        r.process(O.BatchArrays(kid, [price, vol], [2, 2]))
    recs = [(f"S{kid[i]}", StockEvent(f"S{kid[i]}", int(price[i]), int(vol[i])), "stock-events", 0, i, i)
            for i in range(n)]
    want = [(recs[m.record][0], seq_view(sequence_from_traversal(
        m.traversal, p.names, lambda i: Ev(recs[i][0], recs[i][1], i, "stock-events", 0, i))))
        for m in r.matches(with_groups=False) if m.record < oe.value.record]
    got = []
    proc = GpuCEPProcessor("Stocks", PL.stock_demo(), STOCK_SCHEMA, stock_columns(), batch_size=n)
    proc.init(lambda k, s: got.append((k, seq_view(s))))
    with pytest.raises(N.CepError) as ge:
        for rr in recs:
            proc.process(*rr)
    assert (ge.value.code, ge.value.record) == (oe.value.code, oe.value.record)
    assert len(proc.session.batch_errors()[0]) > 1        # several keys failed in the batch
    assert got == want and len(want) > 0


def runs_div_pattern():
    """A runs-path pattern (strict, never branching, a fold) whose second stage divides by (v - 7):
    ArithmeticException on every key that reaches a 7 after its first stage."""
    from kcep import QueryBuilder, Event, States
    return (QueryBuilder().select("a").where(Event.value() > 0).fold("s", Event.value()).then()
            .select("b").where(States.getInt("s") * 100 / (Event.value() - 7) > 10).then()
            .select("c").where(Event.value() > 2).build())


@pytest.mark.parametrize("seed,batch", [(3, 5000), (4, 5000), (5, 2500), (3, 997)])
def test_runs_path_keys_fail_where_the_reference_fails(seed, batch):
    """several keys of one batch throw on the runs path.  cep_batch_errors must list every
    failing key's first exception, so that the processor (which groups a batch by key) fails at the
    first exception in ARRIVAL order and forwards exactly what the reference forwarded before it.
    The failures are constructed, not hoped for: no value is 7 except at five chosen records of five
    keys, all inside one batch, where the strict second stage divides by (v - 7); the first of them in
    arrival order belongs to the largest of the five keys, so the key-grouped batch meets it last."""
    rng = np.random.default_rng(seed)
    n = 5000
    kid = rng.integers(0, 1000, n).astype(np.int32)
    val = rng.integers(1, 200, n).astype(np.int32)
    val[val == 7] = 8
    lo = (n // 2 // batch) * batch                        # one batch: arrival positions [lo, lo + batch)
    hi = min(n, lo + batch)
    pos = []
    for i in range((lo + hi) // 2, hi):                   # records whose key arrived before (run waiting):
        if (kid[:i] == kid[i]).any() and all(kid[j] != kid[i] for j in pos) and \
                (kid[i] > 900 if not pos else kid[i] < kid[pos[0]]):   # the first of a large key
            pos.append(i)
        if len(pos) == 5:
            break
    assert len(pos) == 5
    keys = sorted(int(kid[i]) for i in pos)
    for i in pos:
        val[i] = 7
    sch = Schema([("value", "i32")])
    ir = runs_div_pattern().to_ir(sch)
    assert N.CompiledPattern(ir).info.runs_ok
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, O.MODE_PROCESSOR)
    with pytest.raises(O.OracleError) as oe:
        r.process(O.BatchArrays(kid, [val], [1]))
    assert oe.value.record == pos[0] and kid[pos[0]] == keys[-1]
    recs = [(f"K{kid[i]}", int(val[i]), "t", 0, i, i) for i in range(n)]
    want = [(recs[m.record][0], seq_view(sequence_from_traversal(
        m.traversal, p.names, lambda i: Ev(recs[i][0], recs[i][1], i, "t", 0, i))))
        for m in r.matches(with_groups=False) if m.record < oe.value.record]
    got = []
    proc = GpuCEPProcessor("Div", ir, sch, scalar_column(sch), batch_size=batch)
    proc.init(lambda k, s: got.append((k, seq_view(s))))
    assert proc.session.path == N.PATH_RUNS
    with pytest.raises(N.CepError) as ge:
        for rr in recs:
            proc.process(*rr)
        proc.flush()
    assert (ge.value.code, ge.value.record) == (oe.value.code, oe.value.record) == (5, pos[0])
    assert len(proc.session.batch_errors()[0]) == 5       # every failing key of the batch is listed
    assert got == want and len(want) > 0


def test_record_log_is_pruned_to_carried_events():
    """The host keeps a record only while a carried run can still reach it (positions listed in
    the exported state); pruning must not change the forwarded stream."""
    recs = random_records(99, 25, 3000, 4, null_frac=0.0, redeliver_frac=0.0)
    sch = Schema([("value", "i32")])
    want = oracle_forward(PL.next_one_or_more(), sch, recs)
    proc = GpuCEPProcessor("q", PL.next_one_or_more(), sch, scalar_column(sch), batch_size=32, prune_at=64)
    got = []
    proc.init(lambda k, s: got.append((k, seq_view(s))))
    peak = 0
    for r in recs:
        proc.process(*r)
        peak = max(peak, len(proc._log))
    proc.close()
    assert got == want and len(want) > 0
    assert peak < 600                                     # without pruning it would reach 3000


PROC_FIXTURES = ["proc_high_water_mark", "proc_null_key_value", "integration_multiple_keys",
                 "integration_multiple_topics", "readme_letters", "stock_demo"]


@pytest.mark.parametrize("batch", [1, 100])
@pytest.mark.parametrize("name", PROC_FIXTURES)
def test_every_processor_fixture(name, batch):
    """Every processor-mode golden fixture (CEPProcessorTest, CEPStreamIntegrationTest, README,
    CEPStockDemoTest) through GpuCEPProcessor, records carrying their topic names; sequences
    compared as (stage, [(topic, offset)]) since offsets repeat across topics."""
    fx = fixture(name)
    ev = fx["events"]
    tname = {v: k for k, v in fx["topics"].items()}
    sch = Schema([(c, {1: "i32", 2: "i64", 3: "f64"}[t]) for c, t in fx["columns"]], topics=list(fx["topics"]))
    dec = ColumnDecoder(sch, [lambda v, i=i: v[i] for i in range(len(fx["columns"]))])
    n = len(ev["key"])
    valid = ev.get("valid", [1] * n)
    recs = [(f"k{ev['key'][i]}", tuple(c[i] for c in ev["cols"]) if valid[i] else None, tname[ev["topic"][i]],
             ev["partition"][i], ev["offset"][i], ev["ts"][i]) for i in range(n)]
    got = []
    proc = GpuCEPProcessor(name, bytes.fromhex(fx["ir"]), sch, dec, batch_size=batch)
    proc.init(lambda k, s: got.append([(g.getStage(), [(e.topic, e.offset) for e in g.getEvents()])
                                       for g in s.matched()]))
    for r in recs:
        proc.process(*r)
    proc.close()
    want = [[(g["stage"], [(tname[ev["topic"][i]], ev["offset"][i]) for i in g["events"]]) for g in s]
            for s in fx["expected"]["sequences"]]
    assert got == want
