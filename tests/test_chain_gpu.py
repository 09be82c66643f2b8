"""Parity of the chain path (stencil kernel with optional() stages, CEP_PATH_CHAIN)
with the CPU oracle.

Strict single-cardinality patterns with optional middle stages run on the
streaming stencil kernel with one deterministic run per start record
(compile.cpp analyse_stencil).  Every test calls libkcep.so through the C-ABI on
cuda:0 and compares the emitted matches (emitting record, key and the full
buffer traversal: stage name + record, final stage first) bit-exactly with
oracle/cep_oracle.c on the same seeded inputs."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import synth, Schema, QueryBuilder, Event, Selected
from golden_util import scenarios, event_arrays
from gpu_util import oracle_matches, run_product

pytestmark = pytest.mark.gpu

I32 = Schema([("value", "i32")])


def check(ir, key, cols, coltypes, mode=N.MODE_PROCESSOR, min_matches=1, flags=0, **kw):
    # the device's MODE_NFA is one in-memory NFA per key (the oracle's NFA_PER_KEY)
    omode = O.MODE_PROCESSOR if mode == N.MODE_PROCESSOR else O.MODE_NFA_PER_KEY
    want = oracle_matches(ir, key, cols, coltypes, omode, **kw)
    got, s = run_product(ir, key, cols, mode=mode, flags=flags, **kw)
    assert s.path == N.PATH_CHAIN
    assert got == want
    assert len(got) >= min_matches
    return got


def test_golden_optional_strict():
    """NFATest.java:393-421 (in-memory NFA, one key)."""
    fx = [f for f in scenarios() if f["name"] == "nfa_optional_strict"][0]
    a = event_arrays(fx)
    ir = bytes.fromhex(fx["ir"])
    key = np.zeros_like(a["key"])
    got = check(ir, key, a["cols"], a["coltypes"], mode=fx["mode"], topic=a["topic"], offset=a["offset"],
                ts=a["ts"], flags=N.BATCH_OFFSETS_MONOTONE)
    assert len(got) == len(fx["expected"]["sequences"])


@pytest.mark.parametrize("n,K", [(1, 1), (5, 1), (4099, 7), (50_000, 300), (300_000, 20_000)])
def test_c5_random(n, K):
    rng = np.random.default_rng(n)
    key = np.sort(rng.integers(0, K, n)).astype(np.int32)
    val = rng.integers(0, 64, n).astype(np.int32)
    check(synth.c5_pattern().to_ir(I32), key, [val], [1], min_matches=0 if n < 100 else 1)


def test_c5_generator():
    key, val, _ = synth.c5_stream_np(3000, L=100)
    check(synth.c5_pattern().to_ir(I32), key, [val], [1], min_matches=100)


def _q(stages):
    """stages: [(name, pred, optional)]"""
    q = QueryBuilder()
    for i, (nm, pred, opt) in enumerate(stages):
        if i:
            q = q.then()
        st = q.select(nm)
        if opt:
            st = st.optional()
        q = st.where(pred)
    return q.build()


v = Event.value()
SHAPES = {
    # overlapping predicates: the optional stage and its successor accept the same values
    "overlap": [("a", v == 0, False), ("b", v <= 1, True), ("c", v >= 1, False)],
    # two optionals in a row (a skip can only pass one of them on one record)
    "two_opt": [("a", v == 0, False), ("b", v == 1, True), ("c", v == 2, True), ("d", v <= 2, False)],
    "opt_first_of_four": [("a", v <= 1, False), ("b", v == 1, True), ("c", v != 3, False), ("d", v == 3, False)],
    "dense": [("a", v >= 0, False), ("b", v <= 1, True), ("c", v >= 0, False)],
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("mode", [N.MODE_PROCESSOR, N.MODE_NFA])
def test_shapes(shape, mode):
    rng = np.random.default_rng(len(shape))
    n = 40_000
    key = np.sort(rng.integers(0, 600, n)).astype(np.int32)
    val = rng.integers(0, 4, n).astype(np.int32)
    ir = _q(SHAPES[shape]).to_ir(I32)
    check(ir, key, [val], [1], mode=mode, min_matches=100)


def test_skip_uses_successor_predicate_without_topic():
    """StagesFactory.java:165: SKIP_PROCEED tests the successor's predicate without
    its topic filter; the successor's BEGIN edge still checks the topic."""
    rng = np.random.default_rng(9)
    n = 30_000
    key = np.sort(rng.integers(0, 400, n)).astype(np.int32)
    val = rng.integers(0, 3, n).astype(np.int32)
    topic = rng.integers(0, 2, n).astype(np.int32)
    sch = Schema([("value", "i32")], topics=["t0", "t1"])
    q = (QueryBuilder().select("a").where(Event.value() == 0).then()
         .select("b").optional().where(Event.value() == 1).then()
         .select("c", Selected.withStrictContiguity().withTopic("t1")).where(Event.value() == 2).build())
    check(q.to_ir(sch), key, [val], [1], topic=topic, min_matches=100)


@pytest.mark.parametrize("t", ["i64", "f64"])
def test_wide_columns(t):
    rng = np.random.default_rng(2)
    n = 30_000
    key = np.sort(rng.integers(0, 300, n)).astype(np.int32)
    raw = rng.integers(0, 4, n)
    val = raw.astype(np.int64) * 3_000_000_000 if t == "i64" else raw.astype(np.float64) * 0.25
    c = 3_000_000_000 if t == "i64" else 0.25
    sch = Schema([("value", t)])
    q = (QueryBuilder().select("a").where(Event.value() == 0).then()
         .select("b").optional().where(Event.value() == c).then()
         .select("c").where(Event.value() >= 2 * c).build())
    check(q.to_ir(sch), key, [val], [2 if t == "i64" else 3], min_matches=100)


def test_device_resident_checksum():
    """C5 shape at 10M records: device checksum vs the oracle's (count + hash of every traversal)."""
    import torch
    K = 100_000
    key, val, ts = synth.c5_stream_torch(K, "cuda", L=100)
    ir = synth.c5_pattern().to_ir(I32)
    s = N.Session(N.CompiledPattern(ir), K * 100)
    assert s.path == N.PATH_CHAIN
    s.push(K * 100, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=torch.cuda.current_stream().cuda_stream)
    nm, cs = s.checksum()
    b = O.BatchArrays(key.cpu().numpy(), [val.cpu().numpy()], [1], ts=ts.cpu().numpy())
    assert (nm, cs) == O.baseline(O.OraclePattern(ir), b, O.MODE_PROCESSOR, 16)
    assert nm > 10_000


def test_general_path_still_available():
    """force_path=GENERAL runs the same chain pattern on the NFA kernel, same result."""
    rng = np.random.default_rng(1)
    key = np.sort(rng.integers(0, 100, 5000)).astype(np.int32)
    val = rng.integers(0, 64, 5000).astype(np.int32)
    ir = synth.c5_pattern().to_ir(I32)
    a, _ = run_product(ir, key, [val])
    cp = N.CompiledPattern(ir)
    s = N.Session(cp, len(key), force_path=N.PATH_GENERAL)
    s.push(len(key), key, [val])
    from gpu_util import product_matches
    assert product_matches(s, s.collect()) == a
