"""Host logic of the ingest decoders and GpuCEPProcessor, without a GPU.

* StockEventSerde (example/.../StockEventSerde.java:50-90) on json-simple's wire
  format: HashMap key order, JSONValue.escape, Long-only numeric fields.
* ColumnDecoder narrowing into the schema's column types (Java int/long wrap).
* GpuCEPProcessor's batching around a stand-in session that records what is
  pushed and answers with scripted matches: null filter (CEPProcessor.java:135-138),
  key interning, batches grouped by key for the device, matches forwarded in
  arrival order, truncation at the reference's exception, query-name
  normalisation (:83).  The device side is covered by test_processor_gpu.py.
"""
import numpy as np
import pytest

from kcep import Schema
from kcep import native as N
from kcep.ingest import StockEvent, StockEventSerde, ColumnDecoder, stock_columns, scalar_column
from kcep.processor import GpuCEPProcessor, ProcessorFailed
import patterns_lib as PL


def test_stock_serde_hashmap_order_and_escape():
    # String.hashCode spread into 16 buckets: volume -> 0, price -> 6, name -> 8
    assert StockEventSerde.serialize("t", StockEvent("ALXN", 120, 990)) == b'{"volume":990,"price":120,"name":"ALXN"}'
    assert (StockEventSerde.serialize("t", StockEvent('a/b"c\\\n\u0001 ', -1, 0)) ==
            b'{"volume":0,"price":-1,"name":"a\\/b\\"c\\\\\\n\\u0001\\u2028"}')
    assert StockEventSerde.serialize("t", StockEvent(None, 1, 2)) == b'{"volume":2,"price":1,"name":null}'
    assert StockEventSerde.serialize("t", None) is None


def test_stock_serde_roundtrip_and_errors():
    e = StockEvent("ALXN", 9_000_000_000, -5)
    assert StockEventSerde.deserialize("t", StockEventSerde.serialize("t", e)) == e
    assert StockEventSerde.deserialize("t", None) is None
    with pytest.raises(TypeError, match="ClassCastException"):
        StockEventSerde.deserialize("t", b'{"name":"x","price":1.5,"volume":1}')
    with pytest.raises(TypeError, match="NullPointerException"):
        StockEventSerde.deserialize("t", b'{"name":"x","price":1}')
    with pytest.raises(ValueError):                     # not JSON: RuntimeError(ParseException) in Java
        StockEventSerde.deserialize("t", b'{"name":')


def test_column_decoder_wraps_like_java():
    sch = Schema([("a", "i32"), ("b", "i64"), ("c", "f64")])
    d = ColumnDecoder(sch, [lambda v: v[0], lambda v: v[1], lambda v: v[2]])
    cols = d.columns([d.row((2**31, 2**63, 1)), d.row((-1, -2, 0.5))])
    assert cols[0].dtype == np.int32 and list(cols[0]) == [-2**31, -1]
    assert cols[1].dtype == np.int64 and list(cols[1]) == [-2**63, -2]
    assert cols[2].dtype == np.float64 and list(cols[2]) == [1.0, 0.5]
    s = stock_columns()
    assert s.row(StockEvent("x", 3, 4)) == (3, 4)


class StubSession:
    """Records pushed batches; answers each push with a match for every record whose
    value is in `complete` (traversal = that record alone), plus an optional error."""

    path = N.PATH_GENERAL

    def __init__(self, complete=(), err_value=None):
        self.pos = 0
        self.pushes = []
        self.complete = set(complete)
        self.err_value = err_value
        self.out = None
        self.closed = False

    def stream_position(self):
        return self.pos

    def push(self, n, key, cols, topic=None, partition=None, offset=None, ts=None, flags=0, **kw):
        # the processor hands its batches over in arrival order (CEP_BATCH_ARRIVAL_ORDER): the device groups
        # them and answers in arrival order of the completing record, errors ascending -- as this stub does
        assert flags & N.BATCH_ARRIVAL_ORDER
        self.pushes.append(dict(key=key.copy(), val=cols[0].copy(), offset=offset.copy(), topic=topic.copy()))
        rec, ents = [], []
        err, err_rec = 0, -1
        self.errs, seen = [], set()
        for i in range(n):
            v = int(cols[0][i])
            if v == self.err_value and int(key[i]) not in seen:   # a key stops at its first exception
                seen.add(int(key[i]))
                self.errs.append(self.pos + i)
                if err == 0:
                    err, err_rec = 4, self.pos + i
            if v in self.complete:
                rec.append(self.pos + i)
                ents.append([(0, self.pos + i)])
        self.out = dict(match_record=np.asarray(rec, np.int64), match_key=np.zeros(len(rec), np.int32),
                        ent_off=np.asarray([0] + list(np.cumsum([len(e) for e in ents])), np.int64),
                        ent_name=np.asarray([x[0] for e in ents for x in e], np.int32),
                        ent_record=np.asarray([x[1] for e in ents for x in e], np.int64),
                        path=N.PATH_GENERAL, err=err, err_record=err_rec, msg="NullPointerException")
        self.pos += n

    def collect(self, raise_on_error=True):
        return self.out

    def batch_errors(self):
        return np.asarray(self.errs, np.int64), np.full(len(self.errs), 4, np.int32)

    def close(self):
        self.closed = True


def make(batch, stub):
    sch = Schema([("value", "i32")])
    p = GpuCEPProcessor("My Query\\s+Name", PL.any_any(), sch, scalar_column(sch), batch_size=batch)
    got = []
    p.init(lambda k, s: got.append((k, [(g.getStage(), [e.offset for e in g.getEvents()]) for g in s.matched()])), session=stub)
    return p, got


def test_processor_batches_in_arrival_order_and_forwarded_in_arrival_order():
    stub = StubSession(complete={7})
    p, got = make(6, stub)
    assert p.queryName == "my queryname"               # toLowerCase + literal replace of "\s+"
    recs = [("b", 7, 0), ("a", 1, 1), (None, 7, 2), ("b", None, 3), ("a", 7, 4), ("c", 7, 5), ("b", 7, 6),
            ("c", 2, 7)]
    for k, v, o in recs:
        p.process(k, v, "events", 0, o, 100 + o)
    assert len(stub.pushes) == 1                        # nulls never reach the buffer: 6 records flushed
    b = stub.pushes[0]
    assert list(b["key"]) == [0, 1, 1, 2, 0, 2]         # interned keys, in arrival order (the device groups)
    assert list(b["offset"]) == [0, 1, 4, 5, 6, 7]
    p.close()
    assert stub.closed
    # arrival order of the completing records: 0 (b), 4 (a), 5 (c), 6 (b)
    assert got == [("b", [("$final", [0])]), ("a", [("$final", [4])]), ("c", [("$final", [5])]),
                   ("b", [("$final", [6])])]


def test_processor_error_truncates_and_fails():
    stub = StubSession(complete={7}, err_value=9)
    p, got = make(100, stub)
    for k, v, o in [("a", 7, 0), ("b", 9, 1), ("a", 7, 2), ("c", 7, 3)]:
        p.process(k, v, "events", 0, o, o)
    with pytest.raises(N.CepError) as ei:
        p.punctuate(0)
    assert ei.value.record == 1                          # arrival index of the failing record
    assert got == [("a", [("$final", [0])])]              # only what arrived before it
    with pytest.raises(ProcessorFailed):
        p.process("a", 1, "events", 0, 9, 9)


def test_processor_error_is_first_in_arrival_order():
    """Two keys fail in one batch; the processor must fail where the reference does: at the earliest
    arrival (the device reports the batch's exceptions in arrival order, CEP_BATCH_ARRIVAL_ORDER)."""
    stub = StubSession(complete={7}, err_value=9)
    p, got = make(100, stub)
    for k, v, o in [("a", 7, 0), ("b", 9, 1), ("a", 9, 2), ("a", 7, 3)]:
        p.process(k, v, "events", 0, o, o)
    with pytest.raises(N.CepError) as ei:
        p.flush()
    assert stub.out["err_record"] == 1
    assert ei.value.record == 1 and ei.value.code == 4  # b1 arrived first
    assert got == [("a", [("$final", [0])])]


def test_push_failure_fails_the_processor():
    """A push that raises (e.g. CEP_E_RUN_CAPACITY) leaves the batch uncommitted on the device:
    the processor must be failed, not silently drop the batch and carry on."""
    class Boom(StubSession):
        def push(self, *a, **kw):
            raise N.CepError(9, "a key exceeded the largest NFA workspace")
    p, got = make(2, Boom())
    p.process("a", 1, "events", 0, 0, 0)
    with pytest.raises(N.CepError):
        p.process("a", 2, "events", 0, 1, 1)
    with pytest.raises(ProcessorFailed):
        p.process("a", 3, "events", 0, 2, 2)


def test_restore_reseeds_topic_ids():
    """checkpoint() carries the Schema's topic ids; restore() into a fresh schema adopts them and
    refuses a schema whose ids already mean other topics (hwm per interned topic id)."""
    class Carry(StubSession):
        def state_export(self, *a):
            return b"KCST"
        def state_clear(self):
            pass
        def state_import(self, blob):
            self.imported = blob
    p, _ = make(100, Carry())
    for t in ("x", "y"):
        p.process("a", 1, t, 0, 0, 0)
    snap = p.checkpoint()
    assert snap["topics"] == {"x": 0, "y": 1}
    sch = Schema([("value", "i32")])
    q = GpuCEPProcessor("q", PL.any_any(), sch, scalar_column(sch))
    q.init(lambda k, s: None, session=Carry())
    q.restore(snap)
    assert sch.topic_id("y") == 1 and sch.topic_id("z") == 2
    sch2 = Schema([("value", "i32")], topics=["y"])
    r = GpuCEPProcessor("q", PL.any_any(), sch2, scalar_column(sch2))
    r.init(lambda k, s: None, session=Carry())
    with pytest.raises(ProcessorFailed):
        r.restore(snap)


def test_carried_positions_parses_export_blob():
    """kcep.processor.carried_positions on a hand-built cep_state_export blob: two keys, the
    first with 1 high-water mark, 2 queued runs and 2 carried events of 1 column."""
    from kcep.processor import carried_positions
    import struct

    def key_words(nhwm, qlen, positions, ncols=1):
        evw = 8 + 2 * ncols
        hdr = [0] * 12
        hdr[3], hdr[4], hdr[5], hdr[10] = nhwm, qlen, len(positions), ncols
        body = [7] * (3 * nhwm + 4 * qlen)
        for p in positions:
            ev = [0] * evw
            ev[0], ev[1] = p & 0xFFFFFFFF, p >> 32
            body += ev
        w = hdr + body
        w[0] = len(w)
        return w

    blob = struct.pack("<IIqi", 0x4B434550, 1, 0, 2)
    for k, ws in ((3, key_words(1, 2, [5, (1 << 33) + 9])), (8, key_words(0, 0, []))):
        blob += struct.pack("<ii", k, len(ws)) + struct.pack(f"<{len(ws)}I", *ws)
    assert carried_positions(blob) == {5, (1 << 33) + 9}
