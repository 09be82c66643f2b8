"""The CPU oracle against the reference's own test vectors (tests/golden/)."""
import pytest

import oracle as O
from golden_util import scenarios, load, event_arrays, seq_repr

SCEN = scenarios()


@pytest.mark.parametrize("fx", SCEN, ids=[f["name"] for f in SCEN])
def test_scenario(fx):
    p = O.OraclePattern(bytes.fromhex(fx["ir"]))
    a = event_arrays(fx)
    b = O.BatchArrays(a["key"], a["cols"], a["coltypes"], valid=a["valid"], topic=a["topic"],
                      partition=a["partition"], offset=a["offset"], ts=a["ts"])
    run = O.OracleRun(p, fx["mode"])
    run.process(b)
    exp = fx["expected"]
    got = [seq_repr(m.groups) for m in run.matches()]
    want = [seq_repr(s) for s in exp["sequences"]]
    assert got == want
    ms = run.matches(with_groups=False)
    if "match_records" in exp:
        assert [m.record for m in ms] == exp["match_records"]
    if "match_keys" in exp:
        assert [m.key for m in ms] == exp["match_keys"]
    if "runs" in exp:
        runs, qs = run.state(0)
        assert (runs, qs) == (exp["runs"], exp["queue"])
    if "queue_entries" in exp:
        q = run.queue(0)
        names = p.stages()
        got_q = [dict(stage=names[e["stage"]][0], seq=e["seq"], event=None if e["event"] < 0 else e["event"])
                 for e in q]
        assert got_q == exp["queue_entries"]


SF = load("stages_factory.json")


@pytest.mark.parametrize("fx", SF, ids=[f["name"] for f in SF])
def test_stages_factory(fx):
    exp = fx["expected"]
    if "error" in exp:
        with pytest.raises(O.OracleError) as ei:
            O.OraclePattern(bytes.fromhex(fx["ir"]))
        assert ei.value.code == exp["error"]
        return
    p = O.OraclePattern(bytes.fromhex(fx["ir"]))
    st = p.stages()
    assert len(st) == len(exp["stages"])
    for (name, typ, _w, edges), e in zip(st, exp["stages"]):
        assert name == e["name"] and typ == e["type"]
        if "edges" in e:
            assert [list(x) for x in edges] == e["edges"]
        if "edge_ops" in e:
            assert [op for op, _ in edges][:len(e["edge_ops"])] == e["edge_ops"]
        if "edge_targets" in e:
            assert [st[t][0] for _, t in edges][:len(e["edge_targets"])] == e["edge_targets"]


def test_dewey():
    d = load("dewey.json")
    for v, want in d["to_string"]:
        assert O.dewey_add_stage(v).rsplit(".", 1)[0] == want
    for v, off, want in d["add_run"]:
        assert O.dewey_add_run(v, off) == want
    for v, want in d["add_stage"]:
        assert O.dewey_add_stage(v) == want
    for v, want in d["add_stage_add_run"]:
        assert O.dewey_add_run(O.dewey_add_stage(v)) == want
    for a, b, want in d["compatible"]:
        assert O.dewey_compatible(a, b) == want


SVB = load("svb.json")


@pytest.mark.parametrize("fx", SVB, ids=[f["name"] for f in SVB])
def test_shared_versioned_buffer(fx):
    """SharedVersionedBufferTest.java:50-87 on the oracle's buffer (put 3/5-arg, get)."""
    from kcep import Schema, QueryBuilder
    from kcep.expr import Event
    # a pattern only to name the stages first / second / latest
    p = O.OraclePattern((QueryBuilder().select("first").where(Event.value() == 0).then()
                         .select("second").where(Event.value() == 1).then()
                         .select("latest").where(Event.value() == 2).build()).to_ir(Schema([("value", "i32")])))
    sid = {name: i for i, (name, _t, _w, _e) in enumerate(p.stages())}
    ev = fx["events"]
    n = len(ev["key"])
    import numpy as np
    b = O.BatchArrays(ev["key"], [np.zeros(n, np.int32)], [1], offset=ev["offset"], ts=ev["ts"])
    run = O.OracleRun(p, O.MODE_NFA_SINGLE)
    run.svb_bind(b)
    for stage, e, prev, pe, ver in fx["puts"]:
        run.svb_put(sid[stage], e, None if prev is None else sid[prev], pe, ver)
    for g in fx["gets"]:
        m = run.svb_get(sid[g["stage"]], g["event"], g["version"])
        groups = dict(m.groups)
        assert sum(len(v) for v in groups.values()) == g["size"]
        for name, evs in g.get("events", {}).items():
            assert groups[name] == evs
        for name, cnt in g.get("counts", {}).items():
            assert len(groups[name]) == cnt
