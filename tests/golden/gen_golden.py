"""Transcribes the reference's own test vectors into JSON fixtures.

Nothing here runs the reference (it is Java and cannot run in this image;
SURVEY.md §8c).  Each scenario below restates one reference test: its pattern
(in the kcep DSL, which mirrors the Java builders), its input records, and the
outputs that test asserts.  Expected values are copied from the cited test
lines; record indices refer to positions in ``events``.

Run:  python tests/golden/gen_golden.py      (writes tests/golden/*.json)
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "kafkastreams-cep_amd"))

from kcep import QueryBuilder, Selected, Schema, TimeUnit, Event, States, Curr, SequenceAgg, Long  # noqa: E402

MODE_NFA_SINGLE, MODE_PROCESSOR = 0, 1


def letter(s):
    return ord(s)


def eq(s):
    """TestMatcher.isEqualTo("A") (core/src/test/.../TestMatcher.java:7-9) on interned letters."""
    return Event.value() == letter(s)


def fixture(name, source, mode, schema, pattern, events, expected, topics=None):
    ir = pattern.to_ir(schema)
    return dict(name=name, source=source, mode=mode,
                columns=[[n, t] for n, t in schema.columns], topics=schema.topics,
                ir=ir.hex(), events=events, expected=expected)


# NFATest events ev1..ev8: keys "ev1".."ev8", values A B C C D C D E, topic "test",
# partition 0, offsets 0..7 (core/src/test/.../nfa/NFATest.java:49-56)
NFA_EV = {f"ev{i + 1}": (i + 1, v, i) for i, v in enumerate("ABCCDCDE")}


def nfa_events(*names):
    ks, vs, offs = [], [], []
    for n in names:
        k, v, off = NFA_EV[n]
        ks.append(k)
        vs.append(letter(v))
        offs.append(off)
    return dict(key=ks, cols=[vs], topic=[0] * len(ks), partition=[0] * len(ks), offset=offs,
                ts=[1_000] * len(ks))


def seq(*groups):
    return [dict(stage=s, events=list(e)) for s, e in groups]


def letters_schema():
    return Schema([("value", "i32")], topics=["test"])


def nfa_fixtures():
    out = []
    S = letters_schema
    # :65-109 testNFAGivenStatefulCondition (values 5,3,4,10; key "key"; topic t1)
    sch = Schema([("value", "i32")], topics=["t1"])
    avg = (States.getInt("sum") / States.getInt("count")).asDouble()
    p = (QueryBuilder().select("first").where(Event.value() > 0)
         .fold("sum", Event.value()).fold("count", 1)
         .then().select("second").oneOrMore().where(avg >= Event.value())
         .fold("sum", Curr.int() + Event.value()).fold("count", Curr.int() + 1)
         .then().select("latest").where(avg < Event.value()).build())
    ev = dict(key=[1] * 4, cols=[[5, 3, 4, 10]], topic=[0] * 4, partition=[0] * 4, offset=[0, 1, 2, 3],
              ts=[1_000] * 4)
    out.append(fixture("nfa_stateful_condition", "NFATest.java:65-109", MODE_NFA_SINGLE, sch, p, ev,
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2]), ("latest", [3]))],
                            runs=5, queue=2)))
    # :111-157 testNFAGivenSequenceCondition
    sch = Schema([("value", "i32")], topics=["t1"])
    p = (QueryBuilder().select("first").where(Event.value() > 0).then()
         .select("second").oneOrMore().where(SequenceAgg.avg() >= Event.value()).then()
         .select("latest").where(SequenceAgg.avg() < Event.value()).build())
    out.append(fixture("nfa_sequence_condition", "NFATest.java:111-157", MODE_NFA_SINGLE, sch, p, ev,
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2]), ("latest", [3]))],
                            runs=5, queue=2)))
    # :165-196 expecting occurrences: A; C{3}; E over ev1 ev3 ev4 ev6 ev8
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").times(3).where(eq("C"))
         .then().select("latest").where(eq("E")).build())
    out.append(fixture("nfa_times3", "NFATest.java:165-196", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev3", "ev4", "ev6", "ev8"),
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2, 3]), ("latest", [4]))],
                            runs=2, queue=1)))
    # :204-232 zeroOrMore, no matching inputs (ev1 ev5)
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").zeroOrMore().where(eq("C"))
         .then().select("latest").where(eq("D")).build())
    out.append(fixture("nfa_zero_or_more_empty", "NFATest.java:204-232", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("latest", [1]))], runs=2, queue=1)))
    # :240-270 zeroOrMore with matching inputs (ev1 ev3 ev4 ev5)
    out.append(fixture("nfa_zero_or_more", "NFATest.java:240-270", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2]), ("latest", [3]))],
                            runs=2, queue=1)))
    # :278-307 times(2).optional(), no matching (ev1 ev5)
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").times(2).optional()
         .where(eq("C")).then().select("latest").where(eq("D")).build())
    out.append(fixture("nfa_optional_times2_empty", "NFATest.java:278-307", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("latest", [1]))], runs=2, queue=1)))
    # :315-346 times(2).optional(), matching (ev1 ev3 ev4 ev5)
    out.append(fixture("nfa_optional_times2", "NFATest.java:315-346", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2]), ("latest", [3]))],
                            runs=2, queue=1)))
    # :354-385 skip-till-next + times(3) (ev1 ev3 ev4 ev5 ev6 ev8)
    p = (QueryBuilder().select("first").where(eq("A")).then()
         .select("second", Selected.withSkipTilNextMatch()).times(3).where(eq("C")).then()
         .select("latest").where(eq("E")).build())
    out.append(fixture("nfa_next_times3", "NFATest.java:354-385", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev3", "ev4", "ev5", "ev6", "ev8"),
                       dict(sequences=[seq(("first", [0]), ("second", [1, 2, 4]), ("latest", [5]))],
                            runs=2, queue=1)))
    # :393-421 optional stage, strict (ev1 ev3)
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").optional().where(eq("B"))
         .then().select("latest").where(eq("C")).build())
    out.append(fixture("nfa_optional_strict", "NFATest.java:393-421", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev3"),
                       dict(sequences=[seq(("first", [0]), ("latest", [1]))], runs=2, queue=1)))
    # :429-457 one run strict (ev1 ev2 ev3)
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").where(eq("B"))
         .then().select("latest").where(eq("C")).build())
    out.append(fixture("nfa_strict3", "NFATest.java:429-457", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3"),
                       dict(sequences=[seq(("first", [0]), ("second", [1]), ("latest", [2]))],
                            runs=2, queue=1)))
    # :465-498 oneOrMore strict (ev1..ev5)
    p = (QueryBuilder().select("firstStage").where(eq("A")).then().select("secondStage").where(eq("B"))
         .then().select("thirdStage").oneOrMore().where(eq("C")).then()
         .select("latestState").where(eq("D")).build())
    out.append(fixture("nfa_one_or_more", "NFATest.java:465-498", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("firstStage", [0]), ("secondStage", [1]), ("thirdStage", [2, 3]),
                                           ("latestState", [4]))], runs=2, queue=1)))
    # :506-532 two consecutive skip-till-next
    p = (QueryBuilder().select("first").where(eq("A")).then()
         .select("second", Selected.withSkipTilNextMatch()).where(eq("C")).then()
         .select("latest", Selected.withSkipTilNextMatch()).where(eq("D")).build())
    out.append(fixture("nfa_next_next", "NFATest.java:506-532", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [2]), ("latest", [4]))], runs=2, queue=1)))
    # :540-567 skip-till-next oneOrMore then skip-till-next
    p = (QueryBuilder().select("first").where(eq("A")).then()
         .select("second", Selected.withSkipTilNextMatch()).oneOrMore().where(eq("C")).then()
         .select("latest", Selected.withSkipTilNextMatch()).where(eq("D")).build())
    out.append(fixture("nfa_next_one_or_more", "NFATest.java:540-567", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [2, 3]), ("latest", [4]))])))
    # :579-615 two consecutive skip-till-any
    p = (QueryBuilder().select("first").where(eq("A")).then()
         .select("second", Selected.withSkipTilAnyMatch()).where(eq("C")).then()
         .select("latest", Selected.withSkipTilAnyMatch()).where(eq("D")).build())
    out.append(fixture("nfa_any_any", "NFATest.java:579-615", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [2]), ("latest", [4])),
                                       seq(("first", [0]), ("second", [3]), ("latest", [4]))],
                            runs=6, queue=4)))
    # :626-672 skip-till-any oneOrMore then strict
    p = (QueryBuilder().select("first").where(eq("A")).then()
         .select("second", Selected.withSkipTilAnyMatch()).oneOrMore().where(eq("C")).then()
         .select("latest").where(eq("D")).build())
    out.append(fixture("nfa_any_one_or_more", "NFATest.java:626-672", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [2, 3]), ("latest", [4])),
                                       seq(("first", [0]), ("second", [2]), ("latest", [4])),
                                       seq(("first", [0]), ("second", [3]), ("latest", [4]))],
                            runs=5, queue=2)))
    # :684-724 strict, strict, any, any
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").where(eq("B")).then()
         .select("three", Selected.withSkipTilAnyMatch()).where(eq("C")).then()
         .select("latest", Selected.withSkipTilAnyMatch()).where(eq("D")).build())
    out.append(fixture("nfa_strict_strict_any_any", "NFATest.java:684-724", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [1]), ("three", [2]), ("latest", [4])),
                                       seq(("first", [0]), ("second", [1]), ("three", [3]), ("latest", [4]))],
                            runs=6, queue=4)))
    # :732-772 multiple strategies: any then next
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").where(eq("B")).then()
         .select("three", Selected.withSkipTilAnyMatch()).where(eq("C")).then()
         .select("latest", Selected.withSkipTilNextMatch()).where(eq("D")).build())
    out.append(fixture("nfa_multiple_strategies", "NFATest.java:732-772", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev4", "ev5"),
                       dict(sequences=[seq(("first", [0]), ("second", [1]), ("three", [2]), ("latest", [4])),
                                       seq(("first", [0]), ("second", [1]), ("three", [3]), ("latest", [4]))],
                            runs=4, queue=2)))
    # :781-834 skip-till-any on the last stage; queue contents asserted at :804-815
    p = (QueryBuilder().select("first").where(eq("A")).then().select("second").where(eq("B")).then()
         .select("three").where(eq("C")).then()
         .select("latest", Selected.withSkipTilAnyMatch()).where(eq("D")).build())
    out.append(fixture("nfa_any_on_latest", "NFATest.java:781-834", MODE_NFA_SINGLE, S(), p,
                       nfa_events("ev1", "ev2", "ev3", "ev5", "ev7"),
                       dict(sequences=[seq(("first", [0]), ("second", [1]), ("three", [2]), ("latest", [3])),
                                       seq(("first", [0]), ("second", [1]), ("three", [2]), ("latest", [4]))],
                            runs=4, queue=2,
                            queue_entries=[dict(stage="three", seq=4, event=2),
                                           dict(stage="first", seq=2, event=None)])))
    return out


def stages_factory_fixtures():
    """StagesFactoryTest.java:35-157 (stage tables; no events)."""
    out = []
    sch = Schema([("value", "i32")])
    # :35-45 final oneOrMore -> InvalidPatternException
    p = QueryBuilder().select().oneOrMore().where(Event.value() == 0).build()
    out.append(dict(name="sf_invalid_final_one_or_more", source="StagesFactoryTest.java:35-45",
                    ir=p.to_ir(sch).hex(), expected=dict(error=1)))
    # :47-57 final optional -> InvalidPatternException
    p = QueryBuilder().select().optional().where(Event.value() == 0).build()
    out.append(dict(name="sf_invalid_final_optional", source="StagesFactoryTest.java:47-57",
                    ir=p.to_ir(sch).hex(), expected=dict(error=1)))
    # :59-80 single stage
    p = QueryBuilder().select("stage-1").where(Event.value() == 0).build()
    out.append(dict(name="sf_single", source="StagesFactoryTest.java:59-80", ir=p.to_ir(sch).hex(),
                    expected=dict(stages=[dict(name="$final", type=2, edges=[]),
                                          dict(name="stage-1", type=0, edges=[[0, 0]])])))
    # :82-108 three stages
    p = (QueryBuilder().select("stage-1").where(Event.value() == 0).then()
         .select("stage-2").where(Event.value() % 2 == 0).then()
         .select("stage-3").where(Event.value() > 100).build())
    out.append(dict(name="sf_multiple", source="StagesFactoryTest.java:82-108", ir=p.to_ir(sch).hex(),
                    expected=dict(stages=[dict(name="$final", type=2), dict(name="stage-3", type=1),
                                          dict(name="stage-2", type=1), dict(name="stage-1", type=0)])))
    # :110-157 oneOrMore in the middle
    p = (QueryBuilder().select("stage-1").where(Event.value() == 0).then()
         .select("stage-2").oneOrMore().where(Event.value() % 2 == 0).then()
         .select("stage-3").where(Event.value() > 100).build())
    out.append(dict(name="sf_one_or_more", source="StagesFactoryTest.java:110-157", ir=p.to_ir(sch).hex(),
                    expected=dict(stages=[dict(name="$final", type=2),
                                          dict(name="stage-3", type=1, edge_ops=[0], edge_targets=["$final"]),
                                          dict(name="stage-2", type=1, edge_ops=[1, 2],
                                               edge_targets=["stage-3", "stage-3"]),
                                          dict(name="stage-2", type=1, edge_ops=[0]),
                                          dict(name="stage-1", type=0)])))
    return out


def processor_fixtures():
    out = []
    # CEPProcessorTest.java:93-131: pattern select().where(true); key/value null
    # ignored; offset 0 re-delivered per topic is dropped by the high-water mark.
    sch = Schema([("value", "i32")], topics=["topic-test-1", "topic-test-2"])
    p = QueryBuilder().select().where(True).build()
    ev = dict(key=[1, 2, 1, 2], cols=[[0, 0, 0, 0]], topic=[0, 1, 0, 1], partition=[0] * 4,
              offset=[0, 0, 0, 0], ts=[1, 2, 3, 4])
    out.append(fixture("proc_high_water_mark", "CEPProcessorTest.java:113-131", MODE_PROCESSOR, sch, p, ev,
                       dict(sequences=[seq(("0", [0])), seq(("0", [1]))], match_records=[0, 1])))
    ev = dict(key=[1, 2], cols=[[0, 0]], topic=[0, 0], partition=[0, 0], offset=[0, 1], ts=[1, 2],
              valid=[0, 0])
    out.append(fixture("proc_null_key_value", "CEPProcessorTest.java:93-111", MODE_PROCESSOR, sch, p, ev,
                       dict(sequences=[])))

    # CEPStreamIntegrationTest.java:55-68,117-168 (SIMPLE_PATTERN, keys K1/K2 interleaved)
    sch = Schema([("value", "i32")], topics=["input_topic_1"])
    p = (QueryBuilder().select("stage-1").where(Event.value() == 0).fold("sum", Event.value()).then()
         .select("stage-2").oneOrMore().where(States.getInt("sum") <= 10)
         .fold("sum", Curr.int() + Event.value()).then()
         .select("stage-3").where(States.getInt("sum") + Event.value() > 10)
         .within(1, TimeUnit.HOURS).build())
    K1, K2 = 1, 2
    recs = [(K1, 0), (K2, -10), (K2, 0), (K1, 3), (K2, 6), (K1, 1), (K1, 2), (K1, 6), (K2, 4), (K2, 4)]
    ev = dict(key=[k for k, _ in recs], cols=[[v for _, v in recs]], topic=[0] * 10, partition=[0] * 10,
              offset=list(range(10)), ts=list(range(10)))
    out.append(fixture("integration_multiple_keys", "CEPStreamIntegrationTest.java:117-168", MODE_PROCESSOR,
                       sch, p, ev,
                       dict(sequences=[seq(("stage-1", [0]), ("stage-2", [3, 5, 6]), ("stage-3", [7])),
                                       seq(("stage-1", [2]), ("stage-2", [4, 8]), ("stage-3", [9]))],
                            match_keys=[K1, K2])))

    # CEPStreamIntegrationTest.java:70-83,170-230 (two topics)
    sch = Schema([("value", "i32")], topics=["input_topic_1", "input_topic_2"])
    p = (QueryBuilder().select("stage-1", Selected.withStrictContiguity()).where(Event.value() == 0)
         .fold("sum", Event.value()).then()
         .select("stage-2", Selected.withSkipTilNextMatch().withTopic("input_topic_1")).oneOrMore()
         .where(States.getInt("sum") <= 10).fold("sum", Curr.int() + Event.value()).then()
         .select("stage-3", Selected.withSkipTilAnyMatch().withTopic("input_topic_2"))
         .where(Event.value() >= States.getInt("sum")).within(1, TimeUnit.HOURS).build())
    recs = [(0, 0, 0), (0, 1, 1), (0, 2, 2), (0, 3, 3), (1, 6, 0), (1, 10, 1)]   # (topic, value, offset)
    ev = dict(key=[K1] * 6, cols=[[v for _, v, _ in recs]], topic=[t for t, _, _ in recs], partition=[0] * 6,
              offset=[o for _, _, o in recs], ts=list(range(6)))
    out.append(fixture("integration_multiple_topics", "CEPStreamIntegrationTest.java:170-230", MODE_PROCESSOR,
                       sch, p, ev,
                       dict(sequences=[seq(("stage-1", [0]), ("stage-2", [1, 2, 3]), ("stage-3", [4])),
                                       seq(("stage-1", [0]), ("stage-2", [1, 2, 3]), ("stage-3", [5]))])))

    # CEPStockDemoTest.java:72-138 with Patterns.STOCKS (example/.../Patterns.java:11-25)
    sch = Schema([("price", "i64"), ("volume", "i64")], topics=["stock-events"])
    p = (QueryBuilder().select("stage-1").where(Event.field("volume") > 1000)
         .fold("avg", Event.field("price")).then()
         .select("stage-2", Selected.withSkipTilNextMatch()).zeroOrMore()
         .where(Event.field("price") > States.getLong("avg"))
         .fold("avg", (Curr.long() + Event.field("price")) / 2)
         .fold("volume", Event.field("volume")).then()
         .select("stage-3", Selected.withSkipTilNextMatch())
         .where(Event.field("volume") < 0.8 * States.getOrElse("volume", Long(0)).asLong())
         .within(1, TimeUnit.HOURS).build())
    prices = [100, 120, 120, 121, 120, 125, 120, 120]
    vols = [1010, 990, 1005, 999, 999, 750, 950, 700]
    ev = dict(key=[K1] * 8, cols=[prices, vols], topic=[0] * 8, partition=[0] * 8, offset=list(range(8)),
              ts=list(range(8)))
    out.append(fixture("stock_demo", "CEPStockDemoTest.java:111-138", MODE_PROCESSOR, sch, p, ev,
                       dict(sequences=[seq(("stage-1", [0]), ("stage-2", [1, 2, 3, 4]), ("stage-3", [5])),
                                       seq(("stage-1", [2]), ("stage-2", [3]), ("stage-3", [5])),
                                       seq(("stage-1", [0]), ("stage-2", [1, 2, 3, 4, 5, 6]), ("stage-3", [7])),
                                       seq(("stage-1", [2]), ("stage-2", [3, 5]), ("stage-3", [7]))])))

    # README "Letters" query (README.md:50-62): select-A -> select-B -> select-C (BASELINE C1)
    sch = Schema([("value", "i32")], topics=["Letters"])
    p = (QueryBuilder().select("select-A").where(Event.value() == letter("A")).then()
         .select("select-B").where(Event.value() == letter("B")).then()
         .select("select-C").where(Event.value() == letter("C")).build())
    vals = [letter(c) for c in "ABC"]
    ev = dict(key=[1] * 3, cols=[vals], topic=[0] * 3, partition=[0] * 3, offset=[0, 1, 2], ts=[0, 1, 2])
    out.append(fixture("readme_letters", "README.md:50-62 (BASELINE config C1)", MODE_PROCESSOR, sch, p, ev,
                       dict(sequences=[seq(("select-A", [0]), ("select-B", [1]), ("select-C", [2]))])))
    return out


def dewey_fixtures():
    """DeweyVersionTest.java:24-60 (SharedVersionedBufferTest: svb_fixtures)."""
    return dict(
        name="dewey", source="DeweyVersionTest.java:24-60",
        to_string=[["1", "1"], ["1.0.1", "1.0.1"]],
        add_run=[["1", 1, "2"]],
        add_stage_add_run=[["1", "1.1"]],
        add_stage=[["1", "1.0"]],
        compatible=[["1.0", "2.0", False], ["1.0.0", "1.0", True], ["1.1", "1.0", True], ["1.0", "1.1", False]],
    )


def svb_fixtures():
    """SharedVersionedBufferTest.java:50-87: puts on stages first/second/latest over ev1..ev5
    (keys k1..k5, topic-test partition 0, offsets 0..4, ts 1000000001..5, :38-42) and the
    Sequences the test reads back with buffer.get(Matched.from(stage, ev), version).  A get
    asserts the total size and, per stage name, either the event list or only its size,
    exactly as the Java test does."""
    events = dict(key=[1, 2, 3, 4, 5], offset=[0, 1, 2, 3, 4], ts=[1000000001 + i for i in range(5)])
    one = [["first", 0, None, None, "1"], ["second", 1, "first", 0, "1.0"], ["latest", 2, "second", 1, "1.0.0"]]
    get1 = dict(stage="latest", event=2, version="1.0.0", size=3,
                events={"latest": [2], "second": [1], "first": [0]})
    branch = one + [["second", 2, "second", 1, "1.1"], ["second", 3, "second", 2, "1.1"],
                    ["latest", 4, "second", 3, "1.1.0"]]
    get2 = dict(stage="latest", event=4, version="1.1.0", size=5, counts={"latest": 1, "second": 3, "first": 1})
    return [dict(name="svb_one_run", source="SharedVersionedBufferTest.java:50-62", events=events, puts=one,
                 gets=[get1]),
            dict(name="svb_branching_run", source="SharedVersionedBufferTest.java:64-87", events=events,
                 puts=branch, gets=[get1, get2])]


def main():
    fx = nfa_fixtures() + processor_fixtures()
    with open(os.path.join(HERE, "scenarios.json"), "w") as f:
        json.dump(fx, f, indent=1)
    with open(os.path.join(HERE, "stages_factory.json"), "w") as f:
        json.dump(stages_factory_fixtures(), f, indent=1)
    with open(os.path.join(HERE, "dewey.json"), "w") as f:
        json.dump(dewey_fixtures(), f, indent=1)
    with open(os.path.join(HERE, "svb.json"), "w") as f:
        json.dump(svb_fixtures(), f, indent=1)
    print(f"wrote {len(fx)} scenarios")


if __name__ == "__main__":
    main()
