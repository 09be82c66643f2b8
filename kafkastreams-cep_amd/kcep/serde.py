"""JsonSequenceSerde: host mirror of the reference's JSON output serde.

Reference: ``cep/JsonSequenceSerde.java:58-61`` (``new Gson().toJson(sequence)``)
and ``:80-83`` (``new Gson().fromJson(json, Sequence.class)``). Gson 2.8.2 is not
vendored, so its documented default behaviour is restated here:

* objects: the declared non-static, non-transient fields in declaration order,
  null fields omitted (``serializeNulls`` is off).
  * ``Sequence``: ``matched``, then ``indexed`` (``Sequence.java:38-40``).
  * ``Staged``: ``stage``, ``events`` (``:132-133``).
  * ``Event``: ``key, value, timestamp, topic, partition, offset`` (``Event.java:29-39``).
* ``indexed`` is the ``HashMap`` built by ``Collectors.toMap`` (``Sequence.java:49``). Gson writes
  it in ``HashMap`` iteration order, which ``_java_hashmap_order`` reproduces: ``String.hashCode``,
  the spread ``h ^ (h >>> 16)``, and table doubling from 16 at load factor 0.75.
* strings are escaped the way ``JsonWriter`` escapes them with HTML-safe output on (Gson's
  default): ``< > & = '`` become ``\\u003c`` etc. Doubles are written as
  ``Double.toString`` writes them.
* reading back (``fromJson(..., Sequence.class)``): the generic ``K``/``V`` are erased, so JSON
  numbers come back as ``Double`` (``float``), as ``CEPStreamIntegrationTest.java:144`` notes.
  ``Collection`` fields come back as ``ArrayList``, keeping the JSON order.

The exact bytes are parity-unpinned: the reference tests only compare stage names, values and
topics after a round trip (``CEPStreamIntegrationTest.java:232-255``). ``tests/test_serde.py``
replays those assertions.
"""
from __future__ import annotations

import decimal
import json
import math
from typing import Any, List

from .sequence import Event, Sequence, Staged

_HTML = {"<": "\\u003c", ">": "\\u003e", "&": "\\u0026", "=": "\\u003d", "'": "\\u0027",
         " ": "\\u2028", " ": "\\u2029"}


def _java_string_hash(s: str) -> int:
    """java.lang.String.hashCode over UTF-16 code units, as a signed int32."""
    h = 0
    for cu in s.encode("utf-16-be").hex(" ", 2).split():
        h = (31 * h + int(cu, 16)) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def _java_hashmap_order(keys: List[str]) -> List[str]:
    """Iteration order of a java.util.HashMap filled with `keys` in order
    (default capacity 16, load factor 0.75; bucket lists keep insertion order,
    and a resize split keeps it too)."""
    cap, size = 16, 0
    for _ in keys:
        size += 1
        if size > cap * 3 // 4:
            cap *= 2

    def bucket(k):
        h = _java_string_hash(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)

    return [k for _, _, k in sorted((bucket(k), i, k) for i, k in enumerate(keys))]


def _java_double(x: float) -> str:
    """Double.toString: plain notation for 1e-3 <= |x| < 1e7, else d.dddE[-]n."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    a = abs(x)
    if 1e-3 <= a < 1e7:
        r = repr(x)
        if "e" in r or "E" in r:
            r = format(x, "f")
        return r if "." in r else r + ".0"
    t = decimal.Decimal(repr(a)).as_tuple()         # shortest round-trip digits
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    exp = len(t.digits) + t.exponent - 1
    return ("-" if x < 0 else "") + digits[0] + "." + (digits[1:] or "0") + "E" + str(exp)


def _string(s: str) -> str:
    out = json.dumps(s, ensure_ascii=False)
    return "".join(_HTML.get(c, c) for c in out)


def _value(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return _java_double(v)
    if isinstance(v, str):
        return _string(v)
    if isinstance(v, dict):        # a value object: its fields in declaration (insertion) order
        return "{" + ",".join(_string(str(k)) + ":" + _value(x) for k, x in v.items() if x is not None) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join("null" if x is None else _value(x) for x in v) + "]"
    raise TypeError(f"no JSON mapping for {type(v).__name__}")


def _event(e: Event) -> str:
    parts = []
    for name, v in (("key", e.key), ("value", e.value), ("timestamp", e.timestamp), ("topic", e.topic),
                    ("partition", e.partition), ("offset", e.offset)):
        if v is not None:
            parts.append(_string(name) + ":" + _value(v))
    return "{" + ",".join(parts) + "}"


def _staged(s: Staged) -> str:
    return '{"stage":' + _string(s.stage) + ',"events":[' + ",".join(_event(e) for e in s.getEvents()) + "]}"


class JsonSequenceSerde:
    """Serde<Sequence> with the reference's Gson wire format."""

    @staticmethod
    def serialize(topic: str, sequence: Sequence) -> bytes:
        matched = sequence.matched()
        by_name = {s.stage: s for s in matched}
        indexed = ",".join(_string(k) + ":" + _staged(by_name[k]) for k in _java_hashmap_order(list(by_name)))
        body = '{"matched":[' + ",".join(_staged(s) for s in matched) + '],"indexed":{' + indexed + "}}"
        return body.encode("utf-8")

    @staticmethod
    def deserialize(topic: str, data: bytes) -> Sequence:
        if data is None:
            return None
        doc = json.loads(data.decode("utf-8"))

        def erased(v):                 # Gson's ObjectTypeAdapter for an erased type variable
            if isinstance(v, bool) or v is None or isinstance(v, str):
                return v
            if isinstance(v, (int, float)):
                return float(v)
            if isinstance(v, list):
                return [erased(x) for x in v]
            return {k: erased(x) for k, x in v.items()}

        def staged(d):
            s = _ListStaged(d.get("stage"))
            for e in d.get("events") or []:
                s.events_list.append(Event(erased(e.get("key")), erased(e.get("value")), int(e.get("timestamp", 0)),
                                           e.get("topic"), int(e.get("partition", 0)), int(e.get("offset", 0))))
            return s

        seq = Sequence([staged(d) for d in doc.get("matched") or []])
        seq._indexed = {k: staged(v) for k, v in (doc.get("indexed") or {}).items()}
        return seq


class _ListStaged(Staged):
    """A Staged read back by Gson: its Collection field is an ArrayList in JSON order."""

    def __init__(self, stage):
        super().__init__(stage)
        self.events_list: List[Event] = []

    def getEvents(self):
        return list(self.events_list)
