"""Pattern DSL — the host-side mirror of the reference's query builders.

Same names and argument meaning as the reference Java API:

* ``QueryBuilder.select(...)``            — reference ``cep/pattern/QueryBuilder.java:25-60``
* ``StageBuilder.oneOrMore/zeroOrMore/times`` — ``StageBuilder.java:19-45``
* ``PredicateBuilder.where/optional``     — ``PredicateBuilder.java:19-51``
* ``PatternBuilder.and_/or_/fold/within/then/build`` — ``PatternBuilder.java:21-81``
  (``and``/``or`` are Python keywords, hence the trailing underscore)
* ``Pattern``                             — ``Pattern.java:25-240``
* ``Selected``/``Strategy``                — ``Selected.java:19-67``, ``Strategy.java:22-37``

Predicates are ``kcep.expr`` trees instead of opaque lambdas; that is what
lets ``cep_compile`` lower them onto the GPU.  ``Pattern.to_ir(schema)``
serialises the ancestor chain to the byte IR of ``include/kcep.h``.
"""
from __future__ import annotations

import enum
import struct

from . import expr as X


class Strategy(enum.IntEnum):
    STRICT_CONTIGUITY = 0
    SKIP_TIL_NEXT_MATCH = 1
    SKIP_TIL_ANY_MATCH = 2


class Cardinality(enum.IntEnum):
    ONE = 0
    ONE_OR_MORE = 1


class TimeUnit(enum.Enum):
    MILLISECONDS = 1
    SECONDS = 1000
    MINUTES = 60_000
    HOURS = 3_600_000
    DAYS = 86_400_000

    def toMillis(self, t: int) -> int:
        return int(t) * self.value


class Selected:
    """Selection strategy + optional topic (reference Selected.java:19-67)."""

    def __init__(self, strategy, topic):
        self._strategy = strategy
        self._topic = topic

    @staticmethod
    def withStrictContiguity():
        return Selected(Strategy.STRICT_CONTIGUITY, None)

    @staticmethod
    def withSkipTilAnyMatch():
        return Selected(Strategy.SKIP_TIL_ANY_MATCH, None)

    @staticmethod
    def withSkipTilNextMatch():
        return Selected(Strategy.SKIP_TIL_NEXT_MATCH, None)

    @staticmethod
    def fromTopic(topic: str):
        # strategy stays null: compiling it raises the reference's NPE
        # (Selected.java:48-50 vs StagesFactory.java:106)
        return Selected(None, topic)

    def withTopic(self, topic: str):
        return Selected(self._strategy, topic)

    def withStrategy(self, strategy):
        return Selected(strategy, self._topic)

    def getStrategy(self):
        return self._strategy

    def getTopic(self):
        return self._topic


class StateAggregator:
    """``fold(state, aggregator)`` entry (StateAggregator.java:26-48)."""

    def __init__(self, name: str, aggregate: X.Expr, t=None):
        self.name = name
        self.aggregate = aggregate
        self.t = None if t is None else X.type_code(t)   # None: static type of the bound expression


class Pattern:
    """One link of the ancestor chain (reference Pattern.java)."""

    def __init__(self, level=0, name=None, selected=None, ancestor=None):
        self.level = level
        self.name = name
        self.ancestor = ancestor
        self.aggregates = []
        self.selected = Selected.withStrictContiguity() if selected is None else selected
        self.predicate = None
        self.window_time = None
        self.window_unit = None
        self.cardinality = Cardinality.ONE
        self.is_optional = False
        self.times = 1

    # Pattern.select(...) overloads (Pattern.java:302-320)
    def select(self, name_or_selected=None, selected=None):
        if isinstance(name_or_selected, Selected):
            self.selected = name_or_selected
        elif name_or_selected is not None:
            self.name = name_or_selected
            if selected is not None:
                self.selected = selected
        return StageBuilder(self)

    def andPredicate(self, p):
        self.predicate = p if self.predicate is None else (self.predicate & p)

    def orPredicate(self, p):
        self.predicate = p if self.predicate is None else (self.predicate | p)

    def getName(self):
        return str(self.level) if self.name is None else self.name

    def getAncestor(self):
        return self.ancestor

    def chain(self):
        """Patterns first -> last (the reverse of ``Pattern.iterator``)."""
        out = []
        p = self
        while p is not None:
            out.append(p)
            p = p.ancestor
        return out[::-1]

    def to_ir(self, schema) -> bytes:
        return encode_pattern(self, schema)


class PredicateBuilder:
    def __init__(self, pattern: Pattern):
        self.pattern = pattern

    def where(self, predicate: X.Expr):
        self.pattern.andPredicate(X.lift(predicate))
        return PatternBuilder(self.pattern)

    def optional(self):
        self.pattern.is_optional = True
        return self


class StageBuilder(PredicateBuilder):
    def oneOrMore(self):
        self.pattern.cardinality = Cardinality.ONE_OR_MORE
        return self

    def zeroOrMore(self):
        self.pattern.cardinality = Cardinality.ONE_OR_MORE
        self.pattern.is_optional = True
        return self

    def times(self, n: int):
        self.pattern.times = int(n)
        return self


class PatternBuilder:
    def __init__(self, pattern: Pattern):
        self.pattern = pattern

    def and_(self, predicate):
        self.pattern.andPredicate(X.lift(predicate))
        return self

    def or_(self, predicate):
        self.pattern.orPredicate(X.lift(predicate))
        return self

    def fold(self, state: str, aggregator: X.Expr, t=None):
        """``fold(state, (k, v, curr) -> ...)``.  ``t`` is the boxed result
        type; by default the static type of ``aggregator``."""
        agg = X.lift(aggregator)
        self.pattern.aggregates.append(StateAggregator(state, agg, t))
        return self

    def within(self, time: int, unit: TimeUnit):
        self.pattern.window_time = int(time)
        self.pattern.window_unit = unit
        return self

    def then(self):
        return Pattern(self.pattern.level + 1, None, None, self.pattern)

    def build(self):
        return self.pattern


class QueryBuilder:
    """Entry point (QueryBuilder.java:25-60)."""

    DEFAULT_SELECT_STRATEGY = None

    def select(self, name_or_selected=None, selected=None):
        if isinstance(name_or_selected, Selected):
            return StageBuilder(Pattern(0, None, name_or_selected))
        sel = Selected.withStrictContiguity() if selected is None else selected
        return StageBuilder(Pattern(0, name_or_selected, sel))


# ---------------------------------------------------------------------------
# schema + IR encoding
# ---------------------------------------------------------------------------
class Schema:
    """Typed value columns of the event batch.  ``event.value()`` with no
    name resolves to column 0 (a scalar-valued topic such as
    ``KStream<String, Integer>``)."""

    def __init__(self, columns, topics=None):
        self.columns = [(n, X.type_code(t)) for n, t in columns]
        self.topics = {}
        for t in topics or []:
            self.topic_id(t)

    def resolve(self, name):
        if name is None:
            return 0, self.columns[0][1]
        for i, (n, t) in enumerate(self.columns):
            if n == name:
                return i, t
        raise KeyError(f"unknown column {name!r}")

    def topic_id(self, topic: str) -> int:
        if topic not in self.topics:
            self.topics[topic] = max(self.topics.values(), default=-1) + 1
        return self.topics[topic]


MAGIC = b"KCEP"
IR_VERSION = 1
STRATEGY_NULL = 0xFF


def _put_str(out, s):
    X._put_str(out, s)


def encode_pattern(last: Pattern, schema: Schema) -> bytes:
    """Serialise the ancestor chain ending at ``last`` (the pattern returned
    by ``build()``)."""
    out = bytearray(MAGIC)
    out += struct.pack("<I", IR_VERSION)
    out += struct.pack("<H", len(schema.columns))
    for _, t in schema.columns:
        out.append(t)
    chain = last.chain()
    out += struct.pack("<H", len(chain))
    for p in chain:
        _put_str(out, p.name)
        out += struct.pack("<i", p.level)
        strat = p.selected.getStrategy()
        out.append(STRATEGY_NULL if strat is None else int(strat))
        topic = p.selected.getTopic()
        out += struct.pack("<i", -1 if topic is None else schema.topic_id(topic))
        out.append(int(p.cardinality))
        out.append(1 if p.is_optional else 0)
        out += struct.pack("<i", p.times)
        wms = -1 if p.window_time is None else p.window_unit.toMillis(p.window_time)
        out += struct.pack("<q", wms)
        if p.predicate is None:
            out.append(0)
        else:
            out.append(1)
            X.bind(p.predicate, schema).serialize(out)
        out += struct.pack("<H", len(p.aggregates))
        for a in p.aggregates:
            _put_str(out, a.name)
            bound = X.bind(a.aggregate, schema)
            out.append(bound.t if a.t is None else a.t)
            bound.serialize(out)
    return bytes(out)
