"""JsonSequenceSerde (kcep/serde.py): the Gson wire format of the reference's
output serde, checked the way CEPStreamIntegrationTest.java:144-227 checks it
(serialize, read back with erased generics, compare stage names, values and
topics).  The exact bytes are parity-unpinned (no Gson here); the literal
expectations below restate Gson's documented defaults."""
import json

import numpy as np
import pytest

import oracle as O
from golden_util import scenarios, event_arrays
from kcep.sequence import Event, Sequence, Staged, sequences_from_matches
from kcep.serde import JsonSequenceSerde, _java_double, _java_hashmap_order, _java_string_hash

FX = {f["name"]: f for f in scenarios()}
KEYS = {1: "K1", 2: "K2"}                         # CEPStreamIntegrationTest.java:86-87


def _events(fx):
    a = event_arrays(fx)
    topics = {v: k for k, v in fx["topics"].items()}

    def event_of(r):
        return Event(KEYS[int(a["key"][r])], int(a["cols"][0][r]), int(a["ts"][r]), topics[int(a["topic"][r])],
                     int(a["partition"][r]), int(a["offset"][r]))
    return a, event_of


def _oracle_sequences(fx):
    a, event_of = _events(fx)
    p = O.OraclePattern(bytes.fromhex(fx["ir"]))
    run = O.OracleRun(p, fx["mode"])
    run.process(O.BatchArrays(a["key"], a["cols"], a["coltypes"], topic=a["topic"], partition=a["partition"],
                              offset=a["offset"], ts=a["ts"]))
    out = []
    for m in run.matches():
        seq = Sequence.newBuilder()
        for stage, recs in reversed(m.groups):    # groups are in Sequence order; Builder.build(true) reverses
            for r in recs:
                seq.add(stage, event_of(r))
        out.append((KEYS[m.key], seq.build(True)))
    return out


def _stage_values(seq, stage):
    return [str(e.value) for e in seq.getByName(stage).getEvents()]


def _stage_topics(seq, stage):
    return [e.topic for e in seq.getByName(stage).getEvents()]


def _java_str(v):                                 # Double.toString of the read-back values
    return _java_double(v) if isinstance(v, float) else str(v)


def roundtrip(seq):
    return JsonSequenceSerde.deserialize("out", JsonSequenceSerde.serialize("out", seq))


def test_multiple_keys_roundtrip():
    """CEPStreamIntegrationTest.testPatternGivenMultipleRecordKeys :117-168."""
    res = _oracle_sequences(FX["integration_multiple_keys"])
    assert [k for k, _ in res] == ["K1", "K2"]
    back = [roundtrip(s) for _, s in res]
    want = [{"stage-1": ["0.0"], "stage-2": ["3.0", "1.0", "2.0"], "stage-3": ["6.0"]},
            {"stage-1": ["0.0"], "stage-2": ["6.0", "4.0"], "stage-3": ["4.0"]}]
    for seq, w in zip(back, want):
        assert [seq.getByIndex(i).getStage() for i in range(3)] == ["stage-1", "stage-2", "stage-3"]
        for stage, vals in w.items():
            assert [_java_str(e.value) for e in seq.getByName(stage).getEvents()] == vals


def test_multiple_topics_roundtrip():
    """CEPStreamIntegrationTest.testPatternGivenRecordsFromMultipleTopics :170-227."""
    res = _oracle_sequences(FX["integration_multiple_topics"])
    assert len(res) == 2
    for (k, s), last in zip(res, ["6.0", "10.0"]):
        assert k == "K1"
        seq = roundtrip(s)
        assert [seq.getByIndex(i).getStage() for i in range(3)] == ["stage-1", "stage-2", "stage-3"]
        assert [_java_str(e.value) for e in seq.getByName("stage-1").getEvents()] == ["0.0"]
        assert _stage_topics(seq, "stage-1") == ["input_topic_1"]
        assert [_java_str(e.value) for e in seq.getByName("stage-2").getEvents()] == ["1.0", "2.0", "3.0"]
        assert _stage_topics(seq, "stage-2") == ["input_topic_1"] * 3
        assert [_java_str(e.value) for e in seq.getByName("stage-3").getEvents()] == [last]
        assert _stage_topics(seq, "stage-3") == ["input_topic_2"]


def test_wire_format():
    """Field order, HashMap order of `indexed`, int values as written by Gson."""
    (k, seq), _ = _oracle_sequences(FX["integration_multiple_topics"])
    doc = JsonSequenceSerde.serialize("out", seq).decode()
    ev = '{"key":"K1","value":0,"timestamp":0,"topic":"input_topic_1","partition":0,"offset":0}'
    assert doc.startswith('{"matched":[{"stage":"stage-1","events":[' + ev + "]}")
    assert list(json.loads(doc)["indexed"]) == _java_hashmap_order(["stage-1", "stage-2", "stage-3"])
    assert list(json.loads(doc)) == ["matched", "indexed"]


def test_java_helpers():
    assert _java_string_hash("Aa") == _java_string_hash("BB") == 2112
    assert _java_string_hash("hello") == 99162322
    assert _java_string_hash("stage-1") == -1897529054
    # HashMap buckets at capacity 16: "a"=97 -> 1, "q"=113 -> 1 (insertion order kept), "b" -> 2
    assert _java_hashmap_order(["b", "q", "a"]) == ["q", "a", "b"]
    assert [_java_double(x) for x in (1.0, 10.0, 1e7, 1.5e-4, 0.001, -2.5e20, 3.14)] == \
        ["1.0", "10.0", "1.0E7", "1.5E-4", "0.001", "-2.5E20", "3.14"]


def test_html_escaping():
    s = Sequence([Staged("<a&b='c'>")])
    doc = JsonSequenceSerde.serialize("t", s).decode()
    assert '"stage":"\\u003ca\\u0026b\\u003d\\u0027c\\u0027\\u003e"' in doc


@pytest.mark.gpu
def test_product_csr_to_json():
    """GPU CSR (cep_collect) -> Sequence -> JSON equals the oracle's, record for record."""
    import torch  # noqa: F401
    from kcep import native as N
    fx = FX["integration_multiple_keys"]
    a, event_of = _events(fx)
    order = np.argsort(a["key"], kind="stable")
    cp = N.CompiledPattern(bytes.fromhex(fx["ir"]))
    s = N.Session(cp, len(order), mode=fx["mode"], force_path=N.PATH_GENERAL)
    s.push(len(order), np.ascontiguousarray(a["key"][order]), [np.ascontiguousarray(a["cols"][0][order])],
           topic=np.ascontiguousarray(a["topic"][order]), partition=np.ascontiguousarray(a["partition"][order]),
           offset=np.ascontiguousarray(a["offset"][order]), ts=np.ascontiguousarray(a["ts"][order]))
    out = s.collect()
    got = sequences_from_matches(out, cp.names, lambda r: event_of(int(order[r])))
    want = _oracle_sequences(fx)
    assert [JsonSequenceSerde.serialize("o", q) for _, _, q in got] == \
        [JsonSequenceSerde.serialize("o", q) for _, q in want]
