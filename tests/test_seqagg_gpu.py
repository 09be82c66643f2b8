"""SequenceMatcher reductions beyond avg on the general path against the oracle.

The reference hands the partial Sequence to user code (SequenceMatcher.java:16-38); the reductions
a matcher typically computes over it -- sum, count, min, max over every event or one stage's
events, and a stage's first / last event (Sequence.getByName(stage).getEvents(), a TreeSet) -- are
lowered to OP_SEQ_AGG and evaluated by the device NFA.  Random keyed streams in both modes, plus the
NullPointerException a matcher raises when it asks for a stage the partial sequence lacks."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import QueryBuilder, Selected, Event, SequenceAgg
import patterns_lib as PL
from test_general_gpu import run_both, rand_stream

pytestmark = pytest.mark.gpu

v = Event.value()
PATTERNS = {
    # oneOrMore bounded by the running sum of the whole sequence, closed above the stage's max
    "sum_max": lambda: (QueryBuilder().select("a").where(v == 0).then()
                        .select("b", Selected.withSkipTilNextMatch()).oneOrMore()
                        .where((v > 0) & (SequenceAgg.sum() + v < 12)).then()
                        .select("c", Selected.withSkipTilNextMatch()).where(v >= SequenceAgg.max(stage="b")).build()),
    # skip-till-any: the next stage compares with the first / last event of earlier stages
    "first_last_any": lambda: (QueryBuilder().select("a").where(v < 3).then()
                               .select("b", Selected.withSkipTilAnyMatch()).where(v > SequenceAgg.first(stage="a")).then()
                               .select("c", Selected.withSkipTilAnyMatch())
                               .where((v == SequenceAgg.last(stage="b")) | (v < SequenceAgg.min())).build()),
    # counts per stage and overall
    "count": lambda: (QueryBuilder().select("a").where(v == 1).then()
                      .select("b", Selected.withSkipTilNextMatch()).oneOrMore()
                      .where((v != 1) & (SequenceAgg.count() <= 3)).then()
                      .select("c").where(SequenceAgg.count(stage="b") == v).build()),
}


@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("mode", [O.MODE_PROCESSOR, O.MODE_NFA_PER_KEY], ids=["processor", "nfa"])
@pytest.mark.parametrize("name", list(PATTERNS))
def test_reduction_random(name, mode, interpret):
    key, val = rand_stream(len(name) * 3 + mode, 200, 14, 5)
    ir = PATTERNS[name]().to_ir(PL.I32)
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    oerr = None
    try:
        r.process(O.BatchArrays(key, [val], [1]))
    except O.OracleError as e:                     # the reference's exception (e.g. a traversal of a removed node)
        oerr = (e.code, e.record)
    want = [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]
    cp = N.CompiledPattern(ir)
    gmode = N.MODE_PROCESSOR if mode == O.MODE_PROCESSOR else N.MODE_NFA
    s = N.Session(cp, len(key), mode=gmode, force_path=N.PATH_GENERAL, interpret=interpret)
    assert s.path == N.PATH_GENERAL and s.jit == (not interpret)
    s.push(len(key), key, [val])
    out = s.collect(raise_on_error=False)
    got = []
    for m in range(len(out["match_record"])):
        a, b = out["ent_off"][m], out["ent_off"][m + 1]
        got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                    [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]))
    gerr = (int(out["err"]), int(out["err_record"])) if out["err"] else None
    assert gerr == oerr
    if oerr is not None:                           # what was forwarded before the failing record
        got = [m for m in got if m[0] < oerr[1]]
        want = [m for m in want if m[0] < oerr[1]]
    assert got == want and len(want) > 0


def test_reduction_i64_and_f64_columns():
    """min / max / first over i64 and f64 columns keep the column's type (Math.min / max on doubles)."""
    from kcep import Schema
    sch = Schema([("px", "f64"), ("qty", "i64")])
    p = (QueryBuilder().select("a").where(Event.field("qty") > 0).then()
         .select("b", Selected.withSkipTilNextMatch()).where(Event.field("px") > SequenceAgg.first("px", stage="a")).then()
         .select("c", Selected.withSkipTilNextMatch())
         .where((Event.field("px") < SequenceAgg.max("px")) & (Event.field("qty") >= SequenceAgg.min("qty"))).build())
    rng = np.random.default_rng(5)
    key, _ = rand_stream(8, 150, 12, 4)
    px = np.round(rng.normal(100, 3, len(key)), 2)
    qty = rng.integers(-3, 50, len(key)).astype(np.int64)
    want, got, oerr, gerr = run_both(p.to_ir(sch), O.MODE_PROCESSOR, key, [px, qty], [3, 2])
    assert oerr is None and gerr is None and got == want and len(want) > 0


def test_missing_stage_raises_npe_at_the_same_record():
    """getByName of a stage the partial sequence lacks is null: the matcher's NPE surfaces at the
    record whose evaluation asks for it."""
    p = (QueryBuilder().select("a").where(v == 0).then()
         .select("b").where(v > SequenceAgg.min(stage="nope")).build())
    key, val = rand_stream(3, 40, 10, 3)
    want, got, oerr, gerr = run_both(p.to_ir(PL.I32), O.MODE_PROCESSOR, key, [val], [1])
    assert oerr is not None and oerr[0] == 4 and gerr == oerr and got == want


@pytest.mark.parametrize("lane_nfa", [False, True], ids=["wave", "lane"])
@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
def test_double_sum_and_average_compensated(interpret, lane_nfa):
    """SequenceAgg.sum / avg over a double column are DoubleStream.sum / average: Java 8's compensated
    sum, over the partial sequence in Sequence order (stages in build(true) order, each stage's
    TreeSet ascending).  Magnitudes mixed so that the compensation and the order change results;
    the device must agree with the oracle on every match (tests/test_seqagg_cpu.py pins the
    algorithm by hand)."""
    from kcep import Schema
    sch = Schema([("px", "f64")])
    px = Event.field("px")
    p = (QueryBuilder().select("a").where(px > 1e12).then()
         .select("b", Selected.withSkipTilNextMatch()).oneOrMore().where((px > 0.0) & (px < 1e3)).then()
         .select("c", Selected.withSkipTilNextMatch())
         .where((px < 0.0) & ((SequenceAgg.sum("px") * 7.0 > SequenceAgg.avg("px") * 7.0 * SequenceAgg.count())
                              | (SequenceAgg.sum("px", stage="b") > 1.5))).build())
    rng = np.random.default_rng(11)
    key, _ = rand_stream(21, 120, 12, 4)
    kind = rng.integers(0, 3, len(key))
    val = np.where(kind == 0, rng.choice([1e16, 3e15, 7.1e12], len(key)),
                   np.where(kind == 1, rng.choice([1.0, 0.5, 0.1, 3.3], len(key)), -1.0)).astype(np.float64)
    want, got, oerr, gerr = run_both(p.to_ir(sch), O.MODE_PROCESSOR, key, [val], [3], interpret=interpret,
                                     lane_nfa=lane_nfa)
    assert oerr is None and gerr is None and got == want and len(want) > 0
