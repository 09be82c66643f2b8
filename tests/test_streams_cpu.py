"""kcep/streams.py host logic without a GPU: topic routing, per-topic-partition offsets and the
processor each query gets (the device session replaced by a recording stub)."""
from kcep import QueryBuilder
from kcep.expr import Event
from kcep.streams import ComplexStreamsBuilder, Consumed, Serdes, TopologyTestDriver
from test_processor_cpu import StubSession


def test_builder_routes_topics_and_assigns_offsets():
    b = ComplexStreamsBuilder()
    pat = QueryBuilder().select("a").where(Event.value() == 7).build()
    q1 = b.stream(["t1", "t2"], Consumed.with_(Serdes.String(), Serdes.Integer())).query("Q One", pat)
    q2 = b.stream("t2").query("q2", pat)
    got1 = []
    q1.foreach(lambda k, s: got1.append(k))
    q2.to("out")
    stubs = []

    def factory(proc):
        stubs.append(StubSession(complete={7}))
        return stubs[-1]
    drv = TopologyTestDriver(b.build(), session_factory=factory)
    for t, k, v in [("t1", "x", 7), ("t2", "y", 7), ("t1", "x", 1), ("t3", "z", 7), ("t2", "y", 2)]:
        drv.process(t, k, v)
    k, seq = drv.readOutput("out")                      # flushes every query
    assert k == "y" and drv.readOutput("out") is None
    s1, s2 = stubs
    assert len(s1.pushes) == 1 and len(s2.pushes) == 1
    p1, p2 = s1.pushes[0], s2.pushes[0]
    assert list(p1["key"]) == [0, 1, 0, 1]              # arrival order (the device groups): x, y, x, y
    assert list(p1["offset"]) == [0, 0, 1, 1]           # offsets per (topic, partition)
    assert list(p1["topic"]) == [0, 1, 0, 1]            # source topics interned first: t1=0, t2=1
    assert list(p2["offset"]) == [0, 1] and list(p2["key"]) == [0, 0]
    assert got1 == ["x", "y"]                           # q1's forwards, in arrival order
    drv.close()
