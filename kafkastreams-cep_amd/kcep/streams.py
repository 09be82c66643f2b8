"""``ComplexStreamsBuilder.stream(...).query(...)`` -- the reference's public entry point, on the
device matcher.

Reference: ``cep/ComplexStreamsBuilder.java:31-108`` (``stream(topic | topics | KStream)``),
``cep/CEPStream.java:37-74`` / ``kint/CEPStreamImpl.java:77-95`` (``query(queryName, pattern
[, queried])`` adds one ``CEPProcessor`` per query and returns the ``KStream<K, Sequence<K, V>>`` of
matches).  Here ``query`` attaches a ``GpuCEPProcessor`` (``kcep/processor.py``) instead, and
``TopologyTestDriver`` plays Kafka's ``ProcessorTopologyTestDriver`` the reference's
integration tests use (``CEPStreamIntegrationTest.java:117-230``): ``process(topic, key, value)``
assigns per-topic-partition offsets in process order and ``readOutput(topic)`` returns the next
forwarded ``(key, Sequence)``.

Kafka itself (brokers, consumer groups, changelog topics, serdes on the wire) is out of scope
(SURVEY §2 rows 5b/7/8): records enter through ``process`` with their values already decoded,
and ``Consumed.with_(key_serde, value_decoder)`` names the ``ColumnDecoder`` that turns a value
into the pattern's typed columns.
"""
from __future__ import annotations

from collections import deque
from typing import Any, Callable, Dict, List, Optional, Sequence as Seq, Tuple, Union

from .ingest import ColumnDecoder, scalar_column
from .pattern import Pattern, PatternBuilder, Schema
from .processor import GpuCEPProcessor


class Serdes:
    """Value decoders for scalar topics (Kafka's ``Serdes.Integer()`` etc.): one typed column."""

    @staticmethod
    def Integer() -> ColumnDecoder:
        return scalar_column(Schema([("value", "i32")]))

    @staticmethod
    def Long() -> ColumnDecoder:
        return scalar_column(Schema([("value", "i64")]))

    @staticmethod
    def Double() -> ColumnDecoder:
        return scalar_column(Schema([("value", "f64")]))

    @staticmethod
    def String():
        return None                  # keys are interned as they are; no decoder needed


class Consumed:
    """``Consumed.with(keySerde, valueSerde)``: the value side is a ``ColumnDecoder``."""

    def __init__(self, key_serde=None, value_decoder: Optional[ColumnDecoder] = None):
        self.key_serde = key_serde
        self.value_decoder = value_decoder

    @staticmethod
    def with_(key_serde=None, value_decoder: Optional[ColumnDecoder] = None) -> "Consumed":
        return Consumed(key_serde, value_decoder)


class Queried:
    """``Queried.with(keySerde, valueSerde)`` / ``Queried.as(name)`` (``cep/Queried.java:26-89``):
    the store serdes and name of the reference; kept for API parity (the device holds the state)."""

    def __init__(self, name: Optional[str] = None, key_serde=None, value_serde=None):
        self.name, self.key_serde, self.value_serde = name, key_serde, value_serde

    @staticmethod
    def with_(key_serde=None, value_serde=None) -> "Queried":
        return Queried(None, key_serde, value_serde)

    @staticmethod
    def as_(name: str) -> "Queried":
        return Queried(name)


class KStream:
    """The ``KStream<K, Sequence<K, V>>`` ``query`` returns: forwarded matches go to every sink."""

    def __init__(self):
        self._sinks: List[Callable[[Any, Any], None]] = []

    def foreach(self, fn: Callable[[Any, Any], None]) -> None:
        self._sinks.append(fn)

    def to(self, topic: str, produced=None) -> None:
        self._sinks.append(lambda k, s, t=topic: self._topology._emit(t, k, s))

    def _forward(self, key, seq):
        for f in self._sinks:
            f(key, seq)


class CEPStream:
    """``CEPStream<K, V>`` over one or more source topics (``kint/CEPStreamImpl.java:41-96``)."""

    def __init__(self, topology: "Topology", topics: Seq[str], consumed: Optional[Consumed]):
        self._topology = topology
        self.topics = list(topics)
        self.consumed = consumed or Consumed()

    def query(self, queryName: str, pattern: Union[Pattern, PatternBuilder], queried: Optional[Queried] = None,
              batch_size: int = 1 << 16, device: int = 0, max_keys: int = 1 << 20) -> KStream:
        """Adds the query's processor (``CEPStreamImpl.query`` ``:77-95``); a ``PatternBuilder``
        is built first (``CEPStream.java:37-50``)."""
        if isinstance(pattern, PatternBuilder):
            pattern = pattern.build()
        dec = self.consumed.value_decoder or Serdes.Integer()
        for t in self.topics:                          # source topics get the first topic ids
            dec.schema.topic_id(t)
        proc = GpuCEPProcessor(queryName, pattern, dec.schema, dec, batch_size=batch_size, max_keys=max_keys,
                               device=device)
        out = KStream()
        out._topology = self._topology
        self._topology._add(self.topics, proc, out)
        return out


class Topology:
    def __init__(self):
        self._nodes: List[Tuple[List[str], GpuCEPProcessor, KStream]] = []
        self._outputs: Dict[str, deque] = {}
        self._driver = None

    def _add(self, topics, proc, out):
        self._nodes.append((list(topics), proc, out))

    def _emit(self, topic, key, seq):
        self._outputs.setdefault(topic, deque()).append((key, seq))


class ComplexStreamsBuilder:
    """``ComplexStreamsBuilder`` (``cep/ComplexStreamsBuilder.java:31-108``)."""

    def __init__(self):
        self._topology = Topology()

    def stream(self, topics: Union[str, Seq[str]], consumed: Optional[Consumed] = None) -> CEPStream:
        if isinstance(topics, str):
            topics = [topics]
        return CEPStream(self._topology, topics, consumed)

    def build(self) -> Topology:
        return self._topology


class TopologyTestDriver:
    """In-process driver (Kafka's ``ProcessorTopologyTestDriver`` role): records go to every query
    subscribed to their topic; offsets increase per (topic, partition) in process order.  Output
    is read after a flush, so the processors' batching is invisible to the caller."""

    def __init__(self, topology: Topology, session_factory: Optional[Callable[[GpuCEPProcessor], Any]] = None):
        self.topology = topology
        self._offsets: Dict[Tuple[str, int], int] = {}
        self._clock = 0
        for _topics, proc, out in topology._nodes:
            proc.init(out._forward, session=session_factory(proc) if session_factory else None)

    def process(self, topic: str, key, value, timestamp: Optional[int] = None, partition: int = 0):
        off = self._offsets.get((topic, partition), 0)
        self._offsets[(topic, partition)] = off + 1
        ts = self._clock if timestamp is None else int(timestamp)
        self._clock += 1
        for topics, proc, _out in self.topology._nodes:
            if topic in topics:
                proc.process(key, value, topic, partition, off, ts)

    def readOutput(self, topic: str):
        """Next ``(key, Sequence)`` forwarded to ``topic``, or None."""
        for _topics, proc, _out in self.topology._nodes:
            proc.flush()
        q = self.topology._outputs.get(topic)
        return q.popleft() if q else None

    def close(self):
        for _topics, proc, _out in self.topology._nodes:
            proc.close()
