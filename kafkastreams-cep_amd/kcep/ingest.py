"""Ingest decode: Kafka record values -> typed SoA columns.

The device consumes struct-of-arrays batches (``cep_batch`` in ``include/kcep.h``):
``key_id`` plus typed value columns.  This module holds the host-side decoders
that turn record values into those columns.

* ``StockEvent`` / ``StockEventSerde`` mirror the example application's value type
  and its json-simple serde (``example/.../StockEvent.java:20-41``,
  ``StockEventSerde.java:50-90``).  json-simple 1.1 is not vendored; its
  documented behaviour is restated: ``JSONObject`` is a ``java.util.HashMap`` (so
  ``toJSONString`` writes keys in HashMap iteration order), ``JSONValue.escape``
  escapes ``" \\ /``, ``\\b \\f \\n \\r \\t`` and the ranges U+0000-001F, U+007F-009F,
  U+2000-20FF as upper-case ``\\uXXXX``; integral JSON numbers parse as ``Long``,
  others as ``Double``, so ``(Long) json.get("price")`` throws ``ClassCastException``
  on ``1.5`` and the primitive ``long`` constructor argument throws
  ``NullPointerException`` on a missing field.
* ``ColumnDecoder`` maps a value to the schema's columns with one extractor per
  column; ``stock_columns`` is the one for ``Patterns.STOCKS`` (price, volume).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Callable, List, Optional, Sequence as Seq

import numpy as np

from .pattern import Schema
from .serde import _java_hashmap_order
from .expr import T_I32, T_I64, T_F64

_NP = {T_I32: np.int32, T_I64: np.int64, T_F64: np.float64}
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


@dataclass
class StockEvent:
    """``StockEvent.java:20-30``: name, price (long), volume (long)."""
    name: Optional[str]
    price: int
    volume: int

    def __str__(self):          # StockEvent.toString (:33-40)
        return f"StockEvent{{name='{self.name}', price={self.price}, volume={self.volume}}}"


def _js_escape(s: str) -> str:
    """json-simple ``JSONValue.escape``."""
    out = []
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "/":
            out.append("\\/")
        elif o <= 0x1F or 0x7F <= o <= 0x9F or 0x2000 <= o <= 0x20FF:
            out.append("\\u%04X" % o)
        else:
            out.append(ch)
    return "".join(out)


def _js_value(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    return '"' + _js_escape(str(v)) + '"'


def _parse_int(s: str):
    v = int(s)
    if not (_I64_MIN <= v <= _I64_MAX):       # json-simple: Long.valueOf overflows -> NumberFormatException
        raise ValueError(f"NumberFormatException: For input string: \"{s}\"")
    return v


class StockEventSerde:
    """``StockEventSerde.JsonSerDeserializer`` (``StockEventSerde.java:50-90``)."""

    @staticmethod
    def serialize(topic: str, data: Optional[StockEvent]) -> Optional[bytes]:
        if data is None:
            return None
        fields = {"name": data.name, "price": data.price, "volume": data.volume}
        body = ",".join('"' + _js_escape(k) + '":' + _js_value(fields[k])
                        for k in _java_hashmap_order(list(fields)))
        return ("{" + body + "}").encode("utf-8")

    @staticmethod
    def deserialize(topic: str, data: Optional[bytes]) -> Optional[StockEvent]:
        if data is None:
            return None
        obj = json.loads(data.decode("utf-8"), parse_int=_parse_int, parse_float=float)
        if not isinstance(obj, dict):            # the (JSONObject) cast
            raise TypeError("ClassCastException: not a JSONObject")
        name = obj.get("name")
        if name is not None and not isinstance(name, str):
            raise TypeError("ClassCastException: name is not a String")
        vals = []
        for f in ("price", "volume"):
            v = obj.get(f)
            if v is None:                        # unboxing null into the long parameter
                raise TypeError(f"NullPointerException: {f} is null")
            if isinstance(v, bool) or not isinstance(v, int):
                raise TypeError(f"ClassCastException: {f} is not a Long")
            vals.append(v)
        return StockEvent(name, vals[0], vals[1])


class ColumnDecoder:
    """Value -> the schema's typed columns, one extractor per column.

    ``extractors[i](value)`` returns column i's value; numbers are narrowed the
    way Java narrows them into the column type (``int`` wraps to 32 bits, ``long``
    to 64 bits)."""

    def __init__(self, schema: Schema, extractors: Seq[Callable[[Any], Any]]):
        if len(extractors) != len(schema.columns):
            raise ValueError("one extractor per schema column")
        self.schema = schema
        self.extractors = list(extractors)
        self.dtypes = [_NP[t] for _, t in schema.columns]

    def row(self, value) -> tuple:
        return tuple(f(value) for f in self.extractors)

    def columns(self, rows: List[tuple]) -> List[np.ndarray]:
        """Rows -> contiguous numpy columns (SoA)."""
        out = []
        for i, dt in enumerate(self.dtypes):
            vals = [r[i] for r in rows]
            if dt is np.float64:
                out.append(np.asarray(vals, np.float64))
            else:
                bits = 32 if dt is np.int32 else 64
                mask = (1 << bits) - 1
                wrapped = [((int(v) & mask) ^ (1 << (bits - 1))) - (1 << (bits - 1)) for v in vals]
                out.append(np.asarray(wrapped, dt))
        return out


STOCK_SCHEMA = Schema([("price", "i64"), ("volume", "i64")])


def stock_columns(schema: Schema = STOCK_SCHEMA) -> ColumnDecoder:
    """Columns of ``Patterns.STOCKS`` (``example/.../Patterns.java:11-25``): price, volume."""
    return ColumnDecoder(schema, [lambda e: e.price, lambda e: e.volume])


def scalar_column(schema: Schema, mapping: Optional[Callable[[Any], Any]] = None) -> ColumnDecoder:
    """A scalar-valued topic (``KStream<K, Integer>``), optionally mapped first (for instance
    String letters interned to ints)."""
    return ColumnDecoder(schema, [mapping or (lambda v: v)])
