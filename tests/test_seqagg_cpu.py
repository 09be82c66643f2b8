"""SequenceMatcher reductions on the CPU side: the DSL's lowering rules, the native compiler's
acceptance (cep_compile, no GPU), and the oracle on hand-computed streams.  The reference cannot
run here (no JDK), so these expectations are worked out by hand from Sequence.java / Event.java:
a stage's events form a TreeSet in offset order (one topic/partition), getByName of a missing
stage is null (NullPointerException inside the matcher)."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import QueryBuilder, Selected, Event, SequenceAgg, Schema
import patterns_lib as PL

v = Event.value()


def oracle_run(p, vals, keys=None):
    ir = p.to_ir(PL.I32)
    op = O.OraclePattern(ir)
    r = O.OracleRun(op, O.MODE_PROCESSOR)
    vals = np.asarray(vals, np.int32)
    key = np.zeros(len(vals), np.int32) if keys is None else np.asarray(keys, np.int32)
    err = None
    try:
        r.process(O.BatchArrays(key, [vals], [1]))
    except O.OracleError as e:
        err = (e.code, e.record)
    return [(m.record, [(op.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)], err


def three(pred_c, pred_b=v > 0):
    return (QueryBuilder().select("a").where(v == 0).then().select("b").where(pred_b).then()
            .select("c").where(pred_c).build())


def test_sum_of_a_stage():
    # a@0 b@1(3) c@2: 3 == sum(b) = 3 -> match; a@3 b@4(5) c@5: 4 != 5
    got, err = oracle_run(three(v == SequenceAgg.sum(stage="b")), [0, 3, 3, 0, 5, 4])
    assert err is None and got == [(2, [("c", 2), ("b", 1), ("a", 0)])]


def test_count_min_max_over_every_event():
    # partial sequence at c = {a: v0, b: v1}: count 2, min = 0 (a's value), max = b's value
    got, _ = oracle_run(three(v == SequenceAgg.count()), [0, 7, 2, 0, 1, 3])
    assert [m[0] for m in got] == [2]
    got, _ = oracle_run(three(v == SequenceAgg.max()), [0, 4, 4, 0, 6, 5])
    assert [m[0] for m in got] == [2]
    got, _ = oracle_run(three(v > SequenceAgg.min()), [0, 4, 0, 0, 6, 1])
    assert [m[0] for m in got] == [5]


def test_first_and_last_of_a_one_or_more_stage():
    p = (QueryBuilder().select("a").where(v == 0).then()
         .select("b").oneOrMore().where(v > 0).then()
         .select("c").where((v == SequenceAgg.first(stage="b") * 10) | (v == SequenceAgg.last(stage="b") * 100)).build())
    # b takes 2, 3 (strict oneOrMore), then c: 20 == first(b) * 10
    got, _ = oracle_run(p, [0, 2, 3, 20])
    assert got == [(3, [("c", 3), ("b", 2), ("b", 1), ("a", 0)])]
    got, _ = oracle_run(p, [0, 2, 3, 300])
    assert [m[0] for m in got] == [3]


def test_missing_stage_is_a_null_pointer():
    got, err = oracle_run(three(v > SequenceAgg.max(stage="zzz")), [0, 1, 1])
    assert err == (4, 2)


def test_dsl_rules():
    with pytest.raises(ValueError):
        SequenceAgg.first()                          # first/last read one stage's TreeSet


def java8_double_sum(vals):
    """DoubleStream.sum of Java 8 (Collectors.sumWithCompensation + computeFinalSum: the Kahan sum
    finished as sum + compensation, the simple sum if that is NaN and the simple sum infinite),
    restated from the JDK 8 sources' algorithm for the hand-pinned expectations below."""
    s = c = simple = 0.0
    for d in vals:
        tmp = d - c
        velvel = s + tmp
        c = (velvel - s) - tmp
        s = velvel
        simple += d
    t = s + c
    return simple if (t != t and abs(simple) == float("inf")) else t


def test_double_sum_is_compensated():
    """SequenceAgg.sum over a double column is DoubleStream.sum: compensated.  1e16 + 1.0 + 1.0 in
    Sequence order (a, then b's TreeSet) is 1e16 naively but 1e16 + 2 compensated, so c's predicate
    sum > 1e16 holds.  Parity unpinned by the reference itself (no JVM here): the expectation follows
    JDK 8's summation algorithm (java8_double_sum)."""
    assert java8_double_sum([1e16, 1.0, 1.0]) == 1e16 + 2 and (1e16 + 1.0) + 1.0 == 1e16
    sch = Schema([("px", "f64")])
    px = Event.field("px")
    p = (QueryBuilder().select("a").where(px >= 1e15).then()
         .select("b").oneOrMore().where((px > 0.0) & (px < 10.0)).then()
         .select("c").where((px < 0.0) & (SequenceAgg.sum("px") > 1e16)).build())
    op = O.OraclePattern(p.to_ir(sch))
    vals = np.array([1e16, 1.0, 1.0, -1.0, 1e16, 1.0, -1.0], np.float64)   # second run: 1e16 + 1 -> 1e16
    r = O.OracleRun(op, O.MODE_PROCESSOR)
    r.process(O.BatchArrays(np.zeros(len(vals), np.int32), [vals], [3]))
    got = [m.record for m in r.matches(with_groups=False)]
    assert got == [3]
    # the average over a double column is DoubleStream.average: the same compensated sum / count.
    # run 1: (1e16 + 2) / 3 * 3 > 1e16 (naively 1e16 / 3 * 3 == 1e16, no match); run 2: 1e16 / 2 * 3
    assert java8_double_sum([1e16, 1.0, 1.0]) / 3 * 3.0 > 1e16 and (1e16 + 1.0 + 1.0) / 3 * 3.0 == 1e16
    q = (QueryBuilder().select("a").where(px >= 1e15).then()
         .select("b").oneOrMore().where((px > 0.0) & (px < 10.0)).then()
         .select("c").where((px < 0.0) & (SequenceAgg.avg("px") * 3.0 > 1e16)).build())
    r = O.OracleRun(O.OraclePattern(q.to_ir(sch)), O.MODE_PROCESSOR)
    r.process(O.BatchArrays(np.zeros(len(vals), np.int32), [vals], [3]))
    assert [m.record for m in r.matches(with_groups=False)] == [3, 6]


def test_native_compile_routes_to_general_path():
    cp = N.CompiledPattern(three(v == SequenceAgg.sum(stage="b")).to_ir(PL.I32))
    info = cp.info
    assert info.stencil_ok == 0 and info.chain_ok == 0 and info.runs_ok == 0 and info.n_stages >= 3
