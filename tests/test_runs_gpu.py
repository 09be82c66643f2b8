"""Parity of the deterministic-runs path (csrc/runs.hip, CEP_PATH_RUNS) with the oracle.

Strict patterns whose runs never branch (stateful predicates, folds,
oneOrMore with exclusive TAKE/PROCEED edges, times(n), optional stages) run
one lane per start record.  Every test goes through libkcep.so on cuda:0 and
compares the emitted matches (emitting record, key, full buffer traversal)
and the reference's exception and its record bit-exactly with the oracle."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import synth, Schema, QueryBuilder, Event, States, Curr, Selected, Long
from golden_util import scenarios, event_arrays
import patterns_lib as PL

pytestmark = pytest.mark.gpu

I32 = Schema([("value", "i32")])


def both(ir, key, cols, coltypes, mode=N.MODE_PROCESSOR, interpret=False, **kw):
    omode = O.MODE_PROCESSOR if mode == N.MODE_PROCESSOR else O.MODE_NFA_PER_KEY
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, omode)
    oerr = None
    try:
        r.process(O.BatchArrays(key, cols, coltypes, **kw))
    except O.OracleError as e:
        oerr = (e.code, e.record)
    want = [(m.record, m.key, [(p.names[nm], ev) for nm, ev in m.traversal]) for m in r.matches(with_groups=False)]
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, max(1, len(key)), mode=mode, force_path=N.PATH_RUNS, interpret=interpret)
    assert s.jit == (not interpret)           # compiled-for-the-pattern kernels unless asked otherwise
    s.push(len(key), np.ascontiguousarray(key, np.int32), [np.ascontiguousarray(c) for c in cols],
           flags=N.BATCH_OFFSETS_MONOTONE, **kw)
    out = s.collect(raise_on_error=False)
    assert out["path"] == N.PATH_RUNS
    got = []
    for m in range(len(out["match_record"])):
        a, b = out["ent_off"][m], out["ent_off"][m + 1]
        got.append((int(out["match_record"][m]), int(out["match_key"][m]),
                    [(cp.names[out["ent_name"][i]], int(out["ent_record"][i])) for i in range(a, b)]))
    gerr = (int(out["err"]), int(out["err_record"])) if out["err"] else None
    if oerr is not None:          # the task stops at the first exception: compare what was forwarded
        want = [m for m in want if m[0] < oerr[1]]
        got = [m for m in got if m[0] < oerr[1]]
    return want, got, oerr, gerr


RUNS_FIXTURES = ["nfa_stateful_condition", "nfa_times3", "nfa_optional_times2_empty", "nfa_optional_times2",
                 "nfa_optional_strict", "nfa_strict3", "nfa_one_or_more", "readme_letters"]


@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("name", RUNS_FIXTURES)
def test_golden_runs(name, interpret):
    fx = [f for f in scenarios() if f["name"] == name][0]
    a = event_arrays(fx)
    key = a["key"] if fx["mode"] == O.MODE_PROCESSOR else np.zeros_like(a["key"])
    mode = N.MODE_PROCESSOR if fx["mode"] == O.MODE_PROCESSOR else N.MODE_NFA
    kw = {f: a[f] for f in ("topic", "partition", "offset", "ts") if a[f] is not None}
    want, got, oerr, gerr = both(bytes.fromhex(fx["ir"]), key, a["cols"], a["coltypes"], mode=mode,
                                 interpret=interpret, **kw)
    assert oerr is None and gerr is None
    assert got == want and len(got) == len(fx["expected"]["sequences"])


def walk(n, seed, lo=-5, hi=6):
    return (100 + np.cumsum(np.random.default_rng(seed).integers(lo, hi, n))).astype(np.int32)


@pytest.mark.parametrize("order", ["emit", "window", "radix"])
@pytest.mark.parametrize("nkeys,per_key", [(1, 3000), (300, 40), (5000, 7), (20000, 12)])
def test_c3_stock_random(nkeys, per_key, order, monkeypatch):
    """Every placement of the completed runs: by end chunk straight from runs_sim's results (runs_emit,
    every run shorter than a chunk), the windowed rank (runs_order, every run spanning at most 1024
    records; KCEP_RUNS_EMIT=0 or longer runs) and rocPRIM's radix sort (KCEP_RUNS_RADIX=1, also taken
    by wider batches)."""
    monkeypatch.setenv("KCEP_RUNS_RADIX", "1" if order == "radix" else "0")
    monkeypatch.setenv("KCEP_RUNS_EMIT", "0" if order != "emit" else "1")
    rng = np.random.default_rng(nkeys)
    key = np.repeat(np.arange(nkeys, dtype=np.int32), rng.poisson(per_key, nkeys) + 1)
    val = walk(len(key), nkeys)
    want, got, oerr, gerr = both(PL.c3_stock().to_ir(I32), key, [val], [1])
    assert oerr is None and gerr is None
    assert got == want and len(got) > 10


def test_run_longer_than_the_segment_offsets():
    """A run spanning more records than runs_sim's 12-bit segment offsets hold (4096) sets the segment
    overflow flag: the batch's traversals are then written by walking every completed run again
    (runs_write) -- wider than a chunk too, so the runs are ordered by the radix sort.  Against the
    oracle, next to short runs of other keys."""
    rng = np.random.default_rng(5)
    long_key = np.concatenate([[0], np.ones(5000, np.int32), [2]]).astype(np.int32)
    short = rng.integers(0, 3, 4000).astype(np.int32)
    val = np.concatenate([short[:2000], long_key, short[2000:]])
    key = np.concatenate([np.full(2000, 1), np.full(len(long_key), 2), np.full(2000, 3)]).astype(np.int32)
    ir = (QueryBuilder().select("a").where(Event.value() == 0).then()
          .select("b").oneOrMore().where(Event.value() == 1).then()
          .select("c").where(Event.value() >= 2).build().to_ir(I32))
    want, got, oerr, gerr = both(ir, key, [val], [1])
    assert oerr is None and gerr is None
    assert got == want
    assert any(len(m[2]) == 5002 for m in got)


def test_c3_generator():
    key, val, ts = synth.c3_stream_np(2000, L=100)
    want, got, _, _ = both(synth.c3_pattern().to_ir(I32), key, [val], [1], ts=ts)
    assert got == want and len(got) > 1000


v = Event.value()


def _shapes():
    avg = (States.getLong("s") / States.getLong("c")).asDouble()
    return {
        # oneOrMore with interval-disjoint successor, times(3), optional
        "interval_one_or_more": (QueryBuilder().select("a").where(v == 0).then()
                                 .select("b").oneOrMore().where(v == 1).then()
                                 .select("c").where(v >= 2).build()),
        "times3_then_opt": (QueryBuilder().select("a").where(v <= 1).then()
                            .select("b").times(3).where(v != 3).then()
                            .select("c").optional().where(v == 3).then()
                            .select("d").where(v == 0).build()),
        # long folds (i64) and a double comparison against the running average
        "running_avg": (QueryBuilder().select("first").where(v > 1).fold("s", Event.value().asLong()).fold("c", Long(1))
                        .then().select("mid").oneOrMore().where(avg >= Event.value())
                        .fold("s", Curr.long() + Event.value()).fold("c", Curr.long() + 1).then()
                        .select("last").where(avg < Event.value()).build()),
        # a topic-filtered successor: TAKE and PROCEED exclusive through the topics
        "topics": (QueryBuilder().select("a", Selected.withStrictContiguity().withTopic("t0")).where(v == 0).then()
                   .select("b", Selected.withStrictContiguity().withTopic("t0")).oneOrMore().where(v >= 0).then()
                   .select("c", Selected.withStrictContiguity().withTopic("t1")).where(v >= 0).build()),
    }


@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
@pytest.mark.parametrize("shape", ["interval_one_or_more", "times3_then_opt", "running_avg", "topics"])
@pytest.mark.parametrize("mode", [N.MODE_PROCESSOR, N.MODE_NFA])
def test_shapes(shape, mode, interpret):
    rng = np.random.default_rng(len(shape))
    n = 30_000
    key = np.sort(rng.integers(0, 400, n)).astype(np.int32)
    val = rng.integers(0, 4, n).astype(np.int32) if shape != "running_avg" else walk(n, 3, -2, 3) % 50
    sch = Schema([("value", "i32")], topics=["t0", "t1"])
    pat = _shapes()[shape]
    assert N.CompiledPattern(pat.to_ir(sch)).info.runs_ok
    kw = dict(topic=rng.integers(0, 2, n).astype(np.int32)) if shape == "topics" else {}
    want, got, oerr, gerr = both(pat.to_ir(sch), key, [val.astype(np.int32)], [1], mode=mode, interpret=interpret,
                                 **kw)
    assert oerr is None and gerr is None
    assert got == want and len(got) > 20


@pytest.mark.parametrize("interpret", [False, True], ids=["jit", "interp"])
def test_exceptions_match_the_reference(interpret):
    """The first exception of the batch (here: integer division by zero in a
    stage predicate, and an unset state) and its record are the reference's."""
    a = (QueryBuilder().select("a").where(v >= 0).fold("x", Event.value()).then()
         .select("b").where((States.getInt("x") * 0 + 10) / (Event.value() - 3) > 1).then()
         .select("c").where(States.getInt("nope") > 0).build())
    rng = np.random.default_rng(8)
    key = np.sort(rng.integers(0, 200, 5000)).astype(np.int32)
    val = rng.integers(0, 5, 5000).astype(np.int32)
    want, got, oerr, gerr = both(a.to_ir(I32), key, [val], [1], interpret=interpret)
    assert oerr is not None and gerr == oerr
    assert got == want


def test_c2_and_c5_on_runs_path():
    for pat, vmax in ((synth.c2_pattern(), 4), (synth.c5_pattern(), 64)):
        rng = np.random.default_rng(vmax)
        key = np.sort(rng.integers(0, 3000, 100_000)).astype(np.int32)
        val = rng.integers(0, vmax, 100_000).astype(np.int32)
        want, got, _, _ = both(pat.to_ir(I32), key, [val], [1])
        assert got == want and len(got) > 100


def test_device_resident_checksum_c3():
    """Full C3 shape on device-resident columns: count + order-independent checksum vs the oracle."""
    import torch
    K = 50_000
    key, val, ts = synth.c3_stream_torch(K, "cuda", L=100)
    ir = synth.c3_pattern().to_ir(I32)
    s = N.Session(N.CompiledPattern(ir), K * 100)
    assert s.path == N.PATH_RUNS
    s.push(K * 100, key.data_ptr(), [val.data_ptr()], ts=ts.data_ptr(), mem=N.MEM_DEVICE,
           stream=torch.cuda.current_stream().cuda_stream)
    nm, cs = s.checksum()
    b = O.BatchArrays(key.cpu().numpy(), [val.cpu().numpy()], [1], ts=ts.cpu().numpy())
    assert (nm, cs) == O.baseline(O.OraclePattern(ir), b, O.MODE_PROCESSOR, 16)


@pytest.mark.parametrize("op", ["div", "rem", "div_long"])
def test_integer_division_is_exact(op):
    """The predicates' integer divide (interp.h bc_udiv32: float-reciprocal estimate, two corrections,
    no branch) against Java semantics over the whole int range: quotients and remainders of random
    operands of every magnitude, divisors +-1, MIN_VALUE / -1 (wraps), MIN_VALUE % -1 == 0, and a
    zero divisor (ArithmeticException at its record).  A record matches iff the device's result equals
    the expected column; the expected column is off by one on a third of the records."""
    rng = np.random.default_rng(11)
    n = 60000
    mag = rng.integers(0, 32, n)
    a = (rng.integers(-(2 ** 31), 2 ** 31, n) >> rng.integers(0, 31, n)).astype(np.int64)
    b = (rng.integers(-(2 ** 31), 2 ** 31, n) >> mag).astype(np.int64)
    b[b == 0] = 7
    edge = [(-(2 ** 31), -1), (-(2 ** 31), 1), (2 ** 31 - 1, -1), (-(2 ** 31), -(2 ** 31)), (2 ** 31 - 1, 2 ** 31 - 1),
            (-(2 ** 31), 2 ** 31 - 1), (5, -(2 ** 31)), (-7, 2), (7, -2), (-7, -2), (0, -5), (4294967, 65536)]
    for i, (x, y) in enumerate(edge):
        a[i], b[i] = x, y
    if op == "div_long":                                           # beyond 32 bits: the 64-bit divide
        a[20:60] = rng.integers(-(2 ** 62), 2 ** 62, 40)
        b[40:60] = rng.integers(2 ** 33, 2 ** 40, 20) * rng.choice([-1, 1], 20)
    q = (np.abs(a) // np.abs(b)) * np.sign(a) * np.sign(b)       # truncating, exact in int64
    r = a - q * b                                                  # (MIN_VALUE % -1 == 0)
    if op != "div_long":
        q = np.where((a == -(2 ** 31)) & (b == -1), -(2 ** 31), q)   # Integer.MIN_VALUE / -1 wraps
    want = q if op != "rem" else r
    c = (want + rng.integers(-1, 2, n) * (rng.random(n) < 0.34)).astype(np.int64)
    if op != "div_long":
        c = np.clip(c, -(2 ** 31), 2 ** 31 - 1)
    b[n - 5] = 0                                                   # the task fails there
    key = np.zeros(n, np.int32)
    if op == "div_long":
        sch = Schema([("a", "i64"), ("b", "i64"), ("c", "i64")])
        pred = Event.field("a") / Event.field("b") == Event.field("c")
        cols, types = [a, b, c], [2, 2, 2]
    else:
        sch = Schema([("a", "i32"), ("b", "i32"), ("c", "i32")])
        ex = Event.field("a") / Event.field("b") if op == "div" else Event.field("a") % Event.field("b")
        pred = ex == Event.field("c")
        cols, types = [a.astype(np.int32), b.astype(np.int32), c.astype(np.int32)], [1, 1, 1]
    ir = QueryBuilder().select("s").where(pred).build().to_ir(sch)
    want_m, got, oerr, gerr = both(ir, key, cols, types)
    assert oerr is not None and gerr == oerr and oerr[1] == n - 5
    assert got == want_m and len(got) > n // 2
