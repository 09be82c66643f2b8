"""Patterns of BASELINE.md §3 (C1-C5) and extra shapes used by the parity tests."""
from kcep import QueryBuilder, Selected, Schema, TimeUnit, Event, States, Curr, Long

I32 = Schema([("value", "i32")])


def c3_stock():
    """C3: first v>0 (sum=v, count=1) -> second.oneOrMore (avg >= v; sum+=v, count+=1)
    -> latest (avg < v), within(60 s).  Shape of NFATest.java:66-87."""
    avg = (States.getInt("sum") / States.getInt("count")).asDouble()
    return (QueryBuilder().select("first").where(Event.value() > 0)
            .fold("sum", Event.value()).fold("count", 1).then()
            .select("second").oneOrMore().where(avg >= Event.value())
            .fold("sum", Curr.int() + Event.value()).fold("count", Curr.int() + 1).then()
            .select("latest").where(avg < Event.value()).within(60, TimeUnit.SECONDS).build())


def c4_any():
    """C4: a strict v==0 -> b skip-till-any times(3) v==1 -> c skip-till-any zeroOrMore v==2
    -> d skip-till-any v==3."""
    return (QueryBuilder().select("a").where(Event.value() == 0).then()
            .select("b", Selected.withSkipTilAnyMatch()).times(3).where(Event.value() == 1).then()
            .select("c", Selected.withSkipTilAnyMatch()).zeroOrMore().where(Event.value() == 2).then()
            .select("d", Selected.withSkipTilAnyMatch()).where(Event.value() == 3).build())


def c5_optional():
    """C5: s1 10<=v<20 -> s2.optional() v==5 or v==6 -> s3 (30<=v<40) or v==63, strict."""
    return (QueryBuilder().select("s1").where((Event.value() >= 10) & (Event.value() < 20)).then()
            .select("s2").optional().where((Event.value() == 5) | (Event.value() == 6)).then()
            .select("s3").where(((Event.value() >= 30) & (Event.value() < 40)) | (Event.value() == 63)).build())


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
