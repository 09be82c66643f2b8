"""kcep — MI355X-native drop-in for kafkastreams-cep's NFA evaluation path.

Host-side mirror of the reference's pattern DSL and query entry points; the
matching itself runs in hand-written HIP kernels behind the C-ABI of
``include/kcep.h`` (``libkcep.so``).
"""
from .expr import (Event, States, Curr, SequenceAgg, Int, Long, Double, T_I32, T_I64, T_F64)  # noqa: F401
from .pattern import (QueryBuilder, Pattern, PatternBuilder, StageBuilder, PredicateBuilder,  # noqa: F401
                      Selected, Strategy, Cardinality, TimeUnit, Schema)
from .serde import JsonSequenceSerde  # noqa: F401
from .ingest import StockEvent, StockEventSerde, ColumnDecoder  # noqa: F401
from .processor import GpuCEPProcessor  # noqa: F401

__all__ = [
    "Event", "States", "Curr", "SequenceAgg", "Int", "Long", "Double",
    "QueryBuilder", "Pattern", "PatternBuilder", "StageBuilder", "PredicateBuilder",
    "Selected", "Strategy", "Cardinality", "TimeUnit", "Schema", "JsonSequenceSerde",
    "StockEvent", "StockEventSerde", "ColumnDecoder", "GpuCEPProcessor",
]
