"""Drives the PatternIR natives of jni/kcep_jni.c (compiled unchanged against tests/jni_stub/) the way
java/com/github/fhuss/kafka/streams/cep/pattern/PatternIR.java does -- test infrastructure, no JVM in
the image.

``encode(last, schema)`` restates ``PatternIR.encode`` call for call: the ancestor chain first to last,
``irbSelect(name | null, level, strategy | -1, topic | null)``, ``irbQuantifier``, ``irbWithin``, the
matcher tree in postfix order (``Expr.emit`` of each node kind, ``Matcher.And/Or/NotPredicate``), then
``irbWhere(1)``; per fold the aggregate and ``irbFold(name, type | 0)``; ``irbFinish``, ``irbTopics``,
``irbProbe``.  It walks the Python mirror of the DSL (kcep/pattern.py, kcep/expr.py), whose node kinds
are the Java ``Expr`` kinds one for one:

    kcep.expr                     java .../pattern/ir/Expr.java       builder call
    Const / TrueE / FalseE        Const                               irbConst
    _ColumnRef / Field            Column (value() / field(name))      irbField(schema.column(name))
    _Leaf(OP_EV_TS/OFFSET/...)    EventField                          irbEvent
    TopicEq                       TopicEq (topicIs)                   irbTopicEq(name)
    StateGet / StateGetOrElse     State                               irbState(name, type, orElse)
    FoldCurr                      Curr                                irbCurr
    _SeqAvgRef / _SeqAggRef       Seq                                 irbSeq(kind, column, stage)
    Bin / Un / Cmp / Logic / Not  Bin / Un / Cmp / Logic / Un(NOT)    irbOp
    Cast                          Cast                                irbCast

A leaf that is none of these (``Opaque`` here, a lambda in Java) makes the query a CPU decision.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from jni_twin import JniLib

PFX_IR = "Java_com_github_fhuss_kafka_streams_cep_pattern_PatternIR_"

# every native method of PatternIR.java
NATIVES_IR = ["irbNew", "irbFree", "irbTopic", "irbSelect", "irbQuantifier", "irbWithin", "irbConst", "irbField",
              "irbEvent", "irbTopicEq", "irbState", "irbCurr", "irbSeq", "irbOp", "irbCast", "irbWhere", "irbFold",
              "irbFinish", "irbTopics", "irbProbe", "irbLastError"]

CEP_OK, CEP_E_INVALID_PATTERN, CEP_E_BAD_IR, CEP_E_UNSUPPORTED = 0, 1, 8, 12


class Opaque:
    """A matcher or aggregator PatternIR cannot look into (a Java lambda)."""

    def __init__(self, fn=None):
        self.fn = fn


class _OpaqueLeaf(Exception):
    pass


class _BuilderError(Exception):
    def __init__(self, status, msg):
        super().__init__(msg)
        self.status = status


class IrJni:
    """The PatternIR natives as ctypes calls with the mock JNIEnv of ``JniLib``."""

    def __init__(self, jl: JniLib | None = None):
        self.jl = jl or JniLib()
        L = self.jl.L
        P = C.c_void_p
        i32, i64 = C.c_int32, C.c_int64
        sig = {
            "irbNew": (i64, [P]), "irbFree": (None, [i64]), "irbTopic": (i32, [i64, P]),
            "irbSelect": (i32, [i64, P, i32, i32, P]), "irbQuantifier": (i32, [i64, i32, i32, i32]),
            "irbWithin": (i32, [i64, i64]), "irbConst": (i32, [i64, i32, i64, C.c_double]),
            "irbField": (i32, [i64, i32]), "irbEvent": (i32, [i64, i32]), "irbTopicEq": (i32, [i64, P]),
            "irbState": (i32, [i64, P, i32, i32]), "irbCurr": (i32, [i64, i32]), "irbSeq": (i32, [i64, i32, i32, P]),
            "irbOp": (i32, [i64, i32]), "irbCast": (i32, [i64, i32]), "irbWhere": (i32, [i64, i32]),
            "irbFold": (i32, [i64, P, i32]), "irbFinish": (P, [i64]), "irbTopics": (P, [i64]), "irbProbe": (i32, [P]),
            "irbLastError": (P, []),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, PFX_IR + name)
            f.restype = res
            f.argtypes = [P, P] + args
            setattr(self, "_" + name, f)

    def utf8(self, s):
        """String.getBytes(UTF_8) as a Java byte[] (null for null)."""
        if s is None:
            return None
        return self.jl.arr(np.frombuffer(s.encode("utf-8"), np.int8) if s else np.zeros(0, np.int8))

    def call(self, name, *args):
        return getattr(self, "_" + name)(self.jl.env, None, *args)

    def last_error(self) -> str:
        return self.jl.string(self.call("irbLastError"))


def _check(ij: IrJni, rc):
    if rc != CEP_OK:
        raise _BuilderError(rc, ij.last_error())


def _emit(ij: IrJni, b, e, schema, topic_names):
    """Expr.emit of the node kinds (postfix: children first)."""
    from kcep import expr as X
    call = ij.call
    if isinstance(e, Opaque):
        raise _OpaqueLeaf("opaque matcher")
    if isinstance(e, (X.TrueE, X.FalseE)):
        _check(ij, call("irbConst", b, X.T_BOOL, 1 if isinstance(e, X.TrueE) else 0, 0.0))
    elif isinstance(e, X.Const):
        if e.t == X.T_F64:
            _check(ij, call("irbConst", b, e.t, 0, float(e.v)))
        else:
            _check(ij, call("irbConst", b, e.t, int(e.v), 0.0))
    elif isinstance(e, X._ColumnRef):
        col, _ = schema.resolve(e.name)
        _check(ij, call("irbField", b, col))
    elif isinstance(e, X.Field):
        _check(ij, call("irbField", b, e.col))
    elif isinstance(e, X.TopicEq):
        _check(ij, call("irbTopicEq", b, ij.utf8(topic_names[e.topic_id])))
    elif isinstance(e, X.StateGetOrElse):
        _emit(ij, b, e.default, schema, topic_names)
        _check(ij, call("irbState", b, ij.utf8(e.name), e.t, 1))
    elif isinstance(e, X.StateGet):
        _check(ij, call("irbState", b, ij.utf8(e.name), e.t, 0))
    elif isinstance(e, X.FoldCurr):
        _check(ij, call("irbCurr", b, e.t))
    elif isinstance(e, X._SeqAvgRef):
        col, _ = schema.resolve(e.name)
        _check(ij, call("irbSeq", b, 0, col, None))
    elif isinstance(e, X._SeqAggRef):
        col = 0 if e.kind == X.SEQ_COUNT else schema.resolve(e.name)[0]
        _check(ij, call("irbSeq", b, e.kind, col, ij.utf8(e.stage)))
    elif isinstance(e, (X.Bin, X.Cmp, X.Logic)):
        _emit(ij, b, e.a, schema, topic_names)
        _emit(ij, b, e.b, schema, topic_names)
        _check(ij, call("irbOp", b, e.op))
    elif isinstance(e, (X.Un, X.Not)):
        _emit(ij, b, e.a, schema, topic_names)
        _check(ij, call("irbOp", b, e.op))
    elif isinstance(e, X.Cast):
        _emit(ij, b, e.a, schema, topic_names)
        _check(ij, call("irbCast", b, e.t))
    elif isinstance(e, X._Leaf):
        _check(ij, call("irbEvent", b, e.op))
    else:
        raise _OpaqueLeaf(f"opaque matcher ({type(e).__name__})")


class Lowered:
    def __init__(self, ir=None, topics=(), reason=None, status=0):
        self.ir, self.topics, self.reason, self.status = ir, list(topics), reason, status

    def gpu(self):
        return self.ir is not None


def encode(ij: IrJni, last, schema, pre_topics=None) -> Lowered:
    """PatternIR.encode(last, schema).  ``pre_topics``: the schema's topics before the walk (IrSchema
    .topics(), in id order); by default the schema's current ones."""
    topics_before = list(pre_topics if pre_topics is not None else
                         sorted(schema.topics, key=lambda t: schema.topics[t]))
    chain = last.chain()                                           # first -> last
    types = np.array([t for _, t in schema.columns], np.int32)
    b = ij.call("irbNew", ij.jl.arr(types))
    if b < 0:
        return Lowered(None, (), ij.last_error(), -b)
    names = {i: t for t, i in schema.topics.items()}               # TopicEq ids -> the names Java holds
    try:
        for t in topics_before:
            ij.call("irbTopic", b, ij.utf8(t))
        for p in chain:
            strat = p.selected.getStrategy()
            topic = p.selected.getTopic()
            _check(ij, ij.call("irbSelect", b, ij.utf8(p.name), p.level, -1 if strat is None else int(strat),
                               ij.utf8(topic)))
            _check(ij, ij.call("irbQuantifier", b, int(p.cardinality), 1 if p.is_optional else 0, p.times))
            if p.window_time is not None:
                _check(ij, ij.call("irbWithin", b, p.window_unit.toMillis(p.window_time)))
            if p.predicate is not None:
                _emit(ij, b, p.predicate, schema, names)
                _check(ij, ij.call("irbWhere", b, 1))
            for a in p.aggregates:
                if isinstance(a.aggregate, Opaque):
                    raise _OpaqueLeaf(f"fold '{a.name}' of stage {p.getName()} is an opaque Aggregator")
                _emit(ij, b, a.aggregate, schema, names)
                _check(ij, ij.call("irbFold", b, ij.utf8(a.name), 0 if a.t is None else a.t))
        ir_arr = ij.call("irbFinish", b)
        if not ir_arr:
            return Lowered(None, (), ij.last_error(), -1)
        ir = ij.jl.to_np(ir_arr, np.int8).tobytes()
        tarr = ij.call("irbTopics", b)
        topics = [ij.jl.string(ij.jl.L.mock_obj_get(tarr, i)) for i in range(ij.jl.L.mock_len(tarr))]
        rc = ij.call("irbProbe", ij.jl.arr(np.frombuffer(ir, np.int8)))
        if rc != CEP_OK:
            return Lowered(None, (), ij.last_error(), rc)
        return Lowered(ir, topics, None, CEP_OK)
    except _OpaqueLeaf as o:
        return Lowered(None, (), str(o), -1)
    except _BuilderError as e:
        return Lowered(None, (), str(e), e.status)
    finally:
        ij.call("irbFree", b)
