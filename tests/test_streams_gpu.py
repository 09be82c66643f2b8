"""CEPStreamIntegrationTest (core/src/test/.../CEPStreamIntegrationTest.java:117-230) through the
reference's public entry point, ComplexStreamsBuilder.stream(...).query(...), on the device
(kcep/streams.py), read back with the test driver as the reference's test does."""
import pytest

from kcep import QueryBuilder, Selected, TimeUnit
from kcep.expr import Event, States, Curr
from kcep.streams import ComplexStreamsBuilder, Consumed, Queried, Serdes, TopologyTestDriver

pytestmark = pytest.mark.gpu

INPUT_TOPIC_1, INPUT_TOPIC_2, OUTPUT_TOPIC_1 = "input_topic_1", "input_topic_2", "output_topic_1"
K1, K2 = "K1", "K2"
STAGE_1, STAGE_2, STAGE_3 = "stage-1", "stage-2", "stage-3"

SIMPLE_PATTERN = (QueryBuilder().select(STAGE_1).where(Event.value() == 0).fold("sum", Event.value()).then()
                  .select(STAGE_2).oneOrMore().where(States.getInt("sum") <= 10)
                  .fold("sum", Curr.int() + Event.value()).then()
                  .select(STAGE_3).where(States.getInt("sum") + Event.value() > 10)
                  .within(1, TimeUnit.HOURS).build())

PATTERN_MULTIPLE_TOPICS = (QueryBuilder().select(STAGE_1, Selected.withStrictContiguity()).where(Event.value() == 0)
                           .fold("sum", Event.value()).then()
                           .select(STAGE_2, Selected.withSkipTilNextMatch().withTopic(INPUT_TOPIC_1)).oneOrMore()
                           .where(States.getInt("sum") <= 10).fold("sum", Curr.int() + Event.value()).then()
                           .select(STAGE_3, Selected.withSkipTilAnyMatch().withTopic(INPUT_TOPIC_2))
                           .where(Event.value() >= States.getInt("sum")).within(1, TimeUnit.HOURS).build())


def stages(seq):
    return [seq.getByIndex(i).getStage() for i in range(len(seq.matched()))]


def values(seq, stage):
    return [e.value for e in seq.getByName(stage).getEvents()]


def topics(seq, stage):
    return [e.topic for e in seq.getByName(stage).getEvents()]


@pytest.mark.parametrize("batch", [1, 3, 1 << 16])
def test_pattern_given_multiple_record_keys(batch):
    builder = ComplexStreamsBuilder()
    stream = builder.stream(INPUT_TOPIC_1, Consumed.with_(Serdes.String(), Serdes.Integer()))
    sequences = stream.query("test", SIMPLE_PATTERN, Queried.with_(Serdes.String(), Serdes.Integer()),
                             batch_size=batch)
    sequences.to(OUTPUT_TOPIC_1)
    driver = TopologyTestDriver(builder.build())
    for k, v in [(K1, 0), (K2, -10), (K2, 0), (K1, 3), (K2, 6), (K1, 1), (K1, 2), (K1, 6), (K2, 4), (K2, 4)]:
        driver.process(INPUT_TOPIC_1, k, v)
    results = [driver.readOutput(OUTPUT_TOPIC_1), driver.readOutput(OUTPUT_TOPIC_1)]
    assert driver.readOutput(OUTPUT_TOPIC_1) is None
    (k1, one), (k2, two) = results
    assert k1 == K1 and stages(one) == [STAGE_1, STAGE_2, STAGE_3]
    assert values(one, STAGE_1) == [0] and values(one, STAGE_2) == [3, 1, 2] and values(one, STAGE_3) == [6]
    assert k2 == K2 and stages(two) == [STAGE_1, STAGE_2, STAGE_3]
    assert values(two, STAGE_1) == [0] and values(two, STAGE_2) == [6, 4] and values(two, STAGE_3) == [4]
    driver.close()


@pytest.mark.parametrize("batch", [1, 1 << 16])
def test_pattern_given_records_from_multiple_topics(batch):
    builder = ComplexStreamsBuilder()
    stream = builder.stream([INPUT_TOPIC_1, INPUT_TOPIC_2], Consumed.with_(Serdes.String(), Serdes.Integer()))
    sequences = stream.query("test", PATTERN_MULTIPLE_TOPICS, Queried.with_(Serdes.String(), Serdes.Integer()),
                             batch_size=batch)
    sequences.to(OUTPUT_TOPIC_1)
    driver = TopologyTestDriver(builder.build())
    for t, v in [(INPUT_TOPIC_1, 0), (INPUT_TOPIC_1, 1), (INPUT_TOPIC_1, 2), (INPUT_TOPIC_1, 3),
                 (INPUT_TOPIC_2, 6), (INPUT_TOPIC_2, 10)]:
        driver.process(t, K1, v)
    results = []
    while (r := driver.readOutput(OUTPUT_TOPIC_1)) is not None:
        results.append(r)
    assert len(results) == 2
    for (k, seq), last in zip(results, (6, 10)):
        assert k == K1 and stages(seq) == [STAGE_1, STAGE_2, STAGE_3]
        assert values(seq, STAGE_1) == [0] and topics(seq, STAGE_1) == [INPUT_TOPIC_1]
        assert values(seq, STAGE_2) == [1, 2, 3] and topics(seq, STAGE_2) == [INPUT_TOPIC_1] * 3
        assert values(seq, STAGE_3) == [last] and topics(seq, STAGE_3) == [INPUT_TOPIC_2]
    driver.close()
