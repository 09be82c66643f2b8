"""Predicate / fold expression IR.

The reference's matchers are opaque Java lambdas (``SimpleMatcher.matches``,
``StatefulMatcher.matches``, ``SequenceMatcher.matches`` and
``Aggregator.aggregate``; reference ``cep/pattern/SimpleMatcher.java:32-49``,
``StatefulMatcher.java:29-47``, ``SequenceMatcher.java:16-38``,
``Aggregator.java:27-29``).  A GPU cannot call a lambda, so this module gives
those lambdas an inspectable form: a small typed expression tree with Java
arithmetic semantics (int/long wrap-around, truncating division,
``ArithmeticException`` on integer division by zero, saturating double->int
casts, NaN comparisons false) that serialises to the byte IR consumed by
``cep_compile`` (``include/kcep.h``).

Typing follows Java binary numeric promotion: i32 < i64 < f64.  Booleans are
only produced by comparisons / logic nodes.

Example (NFATest.java:75-78)::

    avg = (States.getInt("sum") / States.getInt("count")).asDouble()
    where(avg >= Event.value())
"""
from __future__ import annotations

import struct

# static types
T_BOOL, T_I32, T_I64, T_F64 = 0, 1, 2, 3
TYPE_NAMES = {T_BOOL: "bool", T_I32: "i32", T_I64: "i64", T_F64: "f64"}
_TYPE_BY_NAME = {"bool": T_BOOL, "i32": T_I32, "int": T_I32, "i64": T_I64,
                 "long": T_I64, "f64": T_F64, "double": T_F64}

# opcodes (must match oracle/cep_oracle.c and csrc/kcep_ir.h)
OP_TRUE = 0x01
OP_FALSE = 0x02
OP_CONST_I32 = 0x03
OP_CONST_I64 = 0x04
OP_CONST_F64 = 0x05
OP_FIELD = 0x10
OP_EV_KEY = 0x11
OP_EV_TS = 0x12
OP_EV_TOPIC_EQ = 0x13
OP_EV_OFFSET = 0x14
OP_EV_PARTITION = 0x15
OP_STATE_GET = 0x20
OP_STATE_GET_OR_ELSE = 0x21
OP_FOLD_CURR = 0x22
OP_SEQ_AVG = 0x23
OP_SEQ_AGG = 0x24
SEQ_SUM, SEQ_COUNT, SEQ_MIN, SEQ_MAX, SEQ_FIRST, SEQ_LAST = 1, 2, 3, 4, 5, 6
OP_NOT = 0x30
OP_AND = 0x31
OP_OR = 0x32
OP_ADD = 0x40
OP_SUB = 0x41
OP_MUL = 0x42
OP_DIV = 0x43
OP_REM = 0x44
OP_NEG = 0x45
OP_EQ = 0x50
OP_NE = 0x51
OP_LT = 0x52
OP_LE = 0x53
OP_GT = 0x54
OP_GE = 0x55
OP_CAST = 0x60

I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1


def type_code(t) -> int:
    if isinstance(t, int):
        return t
    return _TYPE_BY_NAME[t]


def _put_str(out: bytearray, s):
    if s is None:
        out += struct.pack("<H", 0xFFFF)
        return
    b = s.encode("utf-8")
    if len(b) >= 0xFFFF:
        raise ValueError("string too long for IR")
    out += struct.pack("<H", len(b))
    out += b


class Expr:
    """Base of the expression tree.  ``t`` is the static Java type."""

    op = 0
    t = T_BOOL

    def kids(self):
        return ()

    def payload(self, out: bytearray):
        pass

    def serialize(self, out: bytearray):
        out.append(self.op)
        self.payload(out)
        for k in self.kids():
            k.serialize(out)

    # ---- operator sugar (Java semantics) ----
    def __add__(self, o):
        return Bin(OP_ADD, self, lift(o))

    def __radd__(self, o):
        return Bin(OP_ADD, lift(o), self)

    def __sub__(self, o):
        return Bin(OP_SUB, self, lift(o))

    def __rsub__(self, o):
        return Bin(OP_SUB, lift(o), self)

    def __mul__(self, o):
        return Bin(OP_MUL, self, lift(o))

    def __rmul__(self, o):
        return Bin(OP_MUL, lift(o), self)

    def __truediv__(self, o):
        # Java '/': integer division when both sides are integral
        return Bin(OP_DIV, self, lift(o))

    def __rtruediv__(self, o):
        return Bin(OP_DIV, lift(o), self)

    __floordiv__ = __truediv__

    def __mod__(self, o):
        return Bin(OP_REM, self, lift(o))

    def __neg__(self):
        return Un(OP_NEG, self)

    def __eq__(self, o):  # noqa: D401 - builds a node
        return Cmp(OP_EQ, self, lift(o))

    def __ne__(self, o):
        return Cmp(OP_NE, self, lift(o))

    def __lt__(self, o):
        return Cmp(OP_LT, self, lift(o))

    def __le__(self, o):
        return Cmp(OP_LE, self, lift(o))

    def __gt__(self, o):
        return Cmp(OP_GT, self, lift(o))

    def __ge__(self, o):
        return Cmp(OP_GE, self, lift(o))

    def __and__(self, o):
        return Logic(OP_AND, self, lift(o))

    def __or__(self, o):
        return Logic(OP_OR, self, lift(o))

    def __invert__(self):
        return Not(self)

    __hash__ = object.__hash__

    # casts, mirroring Java's (int)/(long)/(double)
    def asInt(self):
        return Cast(self, T_I32)

    def asLong(self):
        return Cast(self, T_I64)

    def asDouble(self):
        return Cast(self, T_F64)

    def to_ir(self) -> bytes:
        out = bytearray()
        self.serialize(out)
        return bytes(out)


def lift(v) -> Expr:
    if isinstance(v, Expr):
        return v
    if isinstance(v, bool):
        return TrueE() if v else FalseE()
    if isinstance(v, int):
        if I32_MIN <= v <= I32_MAX:
            return Const(v, T_I32)
        return Const(v, T_I64)
    if isinstance(v, float):
        return Const(v, T_F64)
    raise TypeError(f"cannot lift {v!r} into an expression")


class TrueE(Expr):
    op = OP_TRUE
    t = T_BOOL


class FalseE(Expr):
    op = OP_FALSE
    t = T_BOOL


class Const(Expr):
    def __init__(self, v, t):
        self.v = v
        self.t = type_code(t)
        self.op = {T_I32: OP_CONST_I32, T_I64: OP_CONST_I64, T_F64: OP_CONST_F64}[self.t]

    def payload(self, out):
        if self.t == T_I32:
            out += struct.pack("<i", int(self.v))
        elif self.t == T_I64:
            out += struct.pack("<q", int(self.v))
        else:
            out += struct.pack("<d", float(self.v))


def Int(v):
    return Const(v, T_I32)


def Long(v):
    return Const(v, T_I64)


def Double(v):
    return Const(float(v), T_F64)


class Field(Expr):
    """A typed value column of the current event (``event.value()`` or
    ``event.value().<field>``)."""
    op = OP_FIELD

    def __init__(self, col: int, t):
        self.col = col
        self.t = type_code(t)

    def payload(self, out):
        out += struct.pack("<H", self.col)


class _Leaf(Expr):
    def __init__(self, op, t):
        self.op = op
        self.t = t


class TopicEq(Expr):
    """``Matcher.TopicPredicate`` (reference Matcher.java:104-120)."""
    op = OP_EV_TOPIC_EQ
    t = T_BOOL

    def __init__(self, topic_id: int):
        self.topic_id = topic_id

    def payload(self, out):
        out += struct.pack("<i", self.topic_id)


class StateGet(Expr):
    """``States.get(name)`` cast to a boxed type (States.java:56-60): throws
    UnknownAggregateException when unset, ClassCastException on type mismatch."""
    op = OP_STATE_GET

    def __init__(self, name: str, t):
        self.name = name
        self.t = type_code(t)

    def payload(self, out):
        out.append(self.t)
        _put_str(out, self.name)


class StateGetOrElse(Expr):
    """``States.getOrElse(name, default)`` (States.java:70-73)."""
    op = OP_STATE_GET_OR_ELSE

    def __init__(self, name: str, default):
        self.name = name
        self.default = lift(default)
        self.t = self.default.t

    def payload(self, out):
        out.append(self.t)
        _put_str(out, self.name)

    def kids(self):
        return (self.default,)


class FoldCurr(Expr):
    """The ``curr`` argument of ``Aggregator.aggregate`` (null -> NPE on use)."""
    op = OP_FOLD_CURR

    def __init__(self, t):
        self.t = type_code(t)

    def payload(self, out):
        out.append(self.t)


class SeqAvg(Expr):
    """``IntSummaryStatistics.getAverage`` over a column of the partial
    sequence that a ``SequenceMatcher`` receives (SequenceMatcher.java:21-26)."""
    op = OP_SEQ_AVG
    t = T_F64

    def __init__(self, col: int):
        self.col = col

    def payload(self, out):
        out += struct.pack("<H", self.col)


class SeqAgg(Expr):
    """A reduction a ``SequenceMatcher`` computes over the partial sequence it receives
    (SequenceMatcher.java:21-26): over every event, or over one stage's events
    (``Sequence.getByName(stage).getEvents()``, a TreeSet in ``Event.compareTo`` order,
    Sequence.java:57-60 / 130-167; a stage missing from the sequence gives null, i.e. a
    NullPointerException in the matcher).  ``sum`` and ``count`` are Java longs
    (``mapToLong(..).sum()``, ``count()``), ``min``/``max`` follow ``Math.min/max``,
    ``first``/``last`` are the TreeSet's ends."""
    op = OP_SEQ_AGG

    def __init__(self, kind: int, col: int, t, stage):
        self.kind, self.col, self.stage = kind, col, stage
        self.t = type_code(t)

    def payload(self, out):
        out.append(self.kind)
        out += struct.pack("<H", self.col)
        _put_str(out, self.stage)


def _promote(a, b):
    if T_BOOL in (a, b):
        raise TypeError("arithmetic on boolean")
    return max(a, b)


class Bin(Expr):
    def __init__(self, op, a: Expr, b: Expr):
        self.op = op
        self.a, self.b = a, b
        self.t = _promote(a.t, b.t)

    def kids(self):
        return (self.a, self.b)


class Un(Expr):
    def __init__(self, op, a: Expr):
        self.op = op
        self.a = a
        if a.t == T_BOOL:
            raise TypeError("negation of boolean")
        self.t = a.t

    def kids(self):
        return (self.a,)


class Cmp(Expr):
    t = T_BOOL

    def __init__(self, op, a: Expr, b: Expr):
        self.op = op
        self.a, self.b = a, b
        if (a.t == T_BOOL) != (b.t == T_BOOL):
            raise TypeError("comparison between boolean and number")
        if a.t == T_BOOL and op not in (OP_EQ, OP_NE):
            raise TypeError("ordering comparison on booleans")

    def kids(self):
        return (self.a, self.b)


class Logic(Expr):
    t = T_BOOL

    def __init__(self, op, a: Expr, b: Expr):
        if a.t != T_BOOL or b.t != T_BOOL:
            raise TypeError("logical operator on non-boolean")
        self.op = op
        self.a, self.b = a, b

    def kids(self):
        return (self.a, self.b)


class Not(Expr):
    op = OP_NOT
    t = T_BOOL

    def __init__(self, a: Expr):
        if a.t != T_BOOL:
            raise TypeError("! on non-boolean")
        self.a = a

    def kids(self):
        return (self.a,)


class Cast(Expr):
    op = OP_CAST

    def __init__(self, a: Expr, t):
        if a.t == T_BOOL:
            raise TypeError("cast of boolean")
        self.a = a
        self.t = type_code(t)

    def payload(self, out):
        out.append(self.t)

    def kids(self):
        return (self.a,)


# ---------------------------------------------------------------------------
# user-facing accessors mirroring the Java lambda arguments
# ---------------------------------------------------------------------------
class _EventNS:
    """``event`` inside a matcher.  Columns are resolved against the schema
    bound when the pattern is compiled (``Schema``)."""

    def value(self, name: str = None):
        return _ColumnRef(name)

    def field(self, name: str):
        return _ColumnRef(name)

    def key(self):
        return _Leaf(OP_EV_KEY, T_I32)

    def timestamp(self):
        return _Leaf(OP_EV_TS, T_I64)

    def offset(self):
        return _Leaf(OP_EV_OFFSET, T_I64)

    def partition(self):
        return _Leaf(OP_EV_PARTITION, T_I32)


class _ColumnRef(Expr):
    """Unresolved column reference; resolved at serialisation time."""
    op = OP_FIELD

    def __init__(self, name):
        self.name = name
        self.t = T_I64  # placeholder numeric type; real type set by bind()

    def payload(self, out):
        raise RuntimeError("unbound column reference (bind a Schema first)")


class _StatesNS:
    def getInt(self, name):
        return StateGet(name, T_I32)

    def getLong(self, name):
        return StateGet(name, T_I64)

    def getDouble(self, name):
        return StateGet(name, T_F64)

    def get(self, name, t="i32"):
        return StateGet(name, t)

    def getOrElse(self, name, default):
        return StateGetOrElse(name, default)


class _CurrNS:
    def int(self):
        return FoldCurr(T_I32)

    def long(self):
        return FoldCurr(T_I64)

    def double(self):
        return FoldCurr(T_F64)


class _SequenceNS:
    """Reductions over the partial ``Sequence`` of a ``SequenceMatcher``: ``avg`` is
    ``IntSummaryStatistics.getAverage`` over every event; the others take an optional stage
    name (``first``/``last`` need one)."""

    def avg(self, name: str = None):
        return _SeqAvgRef(name)

    def sum(self, name: str = None, stage: str = None):
        return _SeqAggRef(SEQ_SUM, name, stage)

    def count(self, stage: str = None):
        return _SeqAggRef(SEQ_COUNT, None, stage)

    def min(self, name: str = None, stage: str = None):
        return _SeqAggRef(SEQ_MIN, name, stage)

    def max(self, name: str = None, stage: str = None):
        return _SeqAggRef(SEQ_MAX, name, stage)

    def first(self, name: str = None, stage: str = None):
        if stage is None:
            raise ValueError("first() needs a stage: Sequence.getByName(stage).getEvents() is the TreeSet it reads")
        return _SeqAggRef(SEQ_FIRST, name, stage)

    def last(self, name: str = None, stage: str = None):
        if stage is None:
            raise ValueError("last() needs a stage: Sequence.getByName(stage).getEvents() is the TreeSet it reads")
        return _SeqAggRef(SEQ_LAST, name, stage)


class _SeqAggRef(Expr):
    op = OP_SEQ_AGG

    def __init__(self, kind, name, stage):
        self.kind, self.name, self.stage = kind, name, stage
        self.t = T_I64  # placeholder numeric type; real type set by bind()

    def payload(self, out):
        raise RuntimeError("unbound sequence column (bind a Schema first)")


class _SeqAvgRef(Expr):
    op = OP_SEQ_AVG
    t = T_F64

    def __init__(self, name):
        self.name = name

    def payload(self, out):
        raise RuntimeError("unbound sequence column (bind a Schema first)")


Event = _EventNS()
States = _StatesNS()
Curr = _CurrNS()
SequenceAgg = _SequenceNS()


def bind(e: Expr, schema) -> Expr:
    """Resolve column references against ``schema`` (returns a new tree)."""
    if isinstance(e, _ColumnRef):
        col, t = schema.resolve(e.name)
        return Field(col, t)
    if isinstance(e, _SeqAvgRef):
        col, _ = schema.resolve(e.name)
        return SeqAvg(col)
    if isinstance(e, _SeqAggRef):
        if e.kind == SEQ_COUNT:
            return SeqAgg(SEQ_COUNT, 0, T_I64, e.stage)
        col, t = schema.resolve(e.name)
        if e.kind == SEQ_SUM:                       # LongStream.sum, or DoubleStream.sum (compensated)
            t = T_F64 if type_code(t) == T_F64 else T_I64
        return SeqAgg(e.kind, col, t, e.stage)
    if isinstance(e, Bin):
        return Bin(e.op, bind(e.a, schema), bind(e.b, schema))
    if isinstance(e, Un):
        return Un(e.op, bind(e.a, schema))
    if isinstance(e, Cmp):
        a, b = bind(e.a, schema), bind(e.b, schema)
        return Cmp(e.op, a, b)
    if isinstance(e, Logic):
        return Logic(e.op, bind(e.a, schema), bind(e.b, schema))
    if isinstance(e, Not):
        return Not(bind(e.a, schema))
    if isinstance(e, Cast):
        return Cast(bind(e.a, schema), e.t)
    if isinstance(e, StateGetOrElse):
        return StateGetOrElse(e.name, bind(e.default, schema))
    return e
