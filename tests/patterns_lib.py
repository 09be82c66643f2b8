"""Patterns of BASELINE.md §3 (C1-C5) and extra shapes used by the parity tests."""
from kcep import QueryBuilder, Selected, Schema, TimeUnit, Event, States, Curr, Long

I32 = Schema([("value", "i32")])


from kcep.synth import c3_pattern as c3_stock, c4_pattern as c4_any, c5_pattern as c5_optional  # noqa: E402,F401


def next_one_or_more():
    return (QueryBuilder().select("first").where(Event.value() == 0).then()
            .select("second", Selected.withSkipTilNextMatch()).oneOrMore().where(Event.value() == 2).then()
            .select("latest", Selected.withSkipTilNextMatch()).where(Event.value() == 3).build())


def any_any():
    return (QueryBuilder().select("first").where(Event.value() == 0).then()
            .select("second", Selected.withSkipTilAnyMatch()).where(Event.value() == 2).then()
            .select("latest", Selected.withSkipTilAnyMatch()).where(Event.value() == 3).build())


def stock_demo():
    """example/.../Patterns.java:11-25 on (price, volume) i64 columns."""
    return (QueryBuilder().select("stage-1").where(Event.field("volume") > 1000)
            .fold("avg", Event.field("price")).then()
            .select("stage-2", Selected.withSkipTilNextMatch()).zeroOrMore()
            .where(Event.field("price") > States.getLong("avg"))
            .fold("avg", (Curr.long() + Event.field("price")) / 2)
            .fold("volume", Event.field("volume")).then()
            .select("stage-3", Selected.withSkipTilNextMatch())
            .where(Event.field("volume") < 0.8 * States.getOrElse("volume", Long(0)).asLong())
            .within(1, TimeUnit.HOURS).build())


STOCK_SCHEMA = Schema([("price", "i64"), ("volume", "i64")])
