"""The Java drop-in's boundary on the GPU: jni/kcep_jni.c (compiled unchanged against
tests/jni_stub/jni.h) driven call for call as java/com/github/fhuss/kafka/streams/cep/processor/GpuCEPProcessor.java drives it
(tests/jni_twin.py), record by record through ``process()`` with flushes every ``batch_size``
records, against the oracle over the same arrival-order stream in processor mode.

* C2 (stencil) and C5 (chain) carry sessions, with re-delivered records: the twin applies the
  high-water mark (CEPProcessor.checkHighWaterMark, CEPProcessor.java:152-160) on the host and
  passes CEP_BATCH_OFFSETS_MONOTONE; the same push with flags = 0 is refused with
  CEP_E_UNSUPPORTED (the round-2 failure).
* A key over the per-key workspace cap is re-pushed with the cap lifted, not dropped.
* More distinct keys than the session's key ids: LRU keys are spilled (cepStateEvict) and
  re-admitted (cepStateImportKeys).
"""
import os

import numpy as np
import pytest

import oracle as O
from kcep import synth
from jni_twin import JniLib, JavaTwin, LIB
import patterns_lib as PL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jl():
    assert os.path.exists(LIB), "build tests/jni_stub first (__graft_entry__.build)"
    return JniLib()


def stream(seed, n_keys, per_key, vmax, redeliver=0.0):
    """Arrival-order records (key, value, offset): keys interleaved as in a topic partition, offsets
    = arrival index; a fraction of records is delivered a second time later (an older offset)."""
    rng = np.random.default_rng(seed)
    key = np.repeat(np.arange(n_keys, dtype=np.int32), rng.poisson(per_key, n_keys) + 1)
    rng.shuffle(key)
    val = rng.integers(0, vmax, len(key)).astype(np.int32)
    off = np.arange(len(key), dtype=np.int64)
    if redeliver:
        dup = np.sort(rng.choice(len(key) - 1, int(len(key) * redeliver), replace=False))
        at = dup + rng.integers(1, 50, len(dup))             # re-delivered a little later
        ins = np.minimum(at, len(key))
        key = np.insert(key, ins, key[dup])
        val = np.insert(val, ins, val[dup])
        off = np.insert(off, ins, off[dup])
    return key, val, off


def oracle_forwards(ir, key, val, off):
    """(key, [(stage, [offsets])]) per match, in forward order: the oracle over the arrival stream."""
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, O.MODE_PROCESSOR)
    r.process(O.BatchArrays(key, [val], [1], offset=off, ts=off))
    out = []
    for m in r.matches(with_groups=False):
        groups = {}
        for nm, pos in m.traversal:
            groups.setdefault(p.names[nm], []).append(int(off[pos]))
        out.append((int(key[m.record]), [(s, sorted(v)) for s, v in reversed(list(groups.items()))]))
    return out


def drive(jl, ir, key, val, off, batch_size, max_keys, **kw):
    t = JavaTwin(jl, ir, [1], batch_size, max_keys, **kw)
    for i in range(len(key)):
        t.process(int(key[i]), [int(val[i])], "events", 0, int(off[i]), int(off[i]))
    t.close()
    return t


@pytest.mark.parametrize("name,mk,vmax,expect_path", [("c2", synth.c2_pattern, 4, 1), ("c5", synth.c5_pattern, 64, 3)])
@pytest.mark.parametrize("batch_size", [1, 7, 4093])
def test_stencil_and_chain_carry_through_jni(jl, name, mk, vmax, expect_path, batch_size):
    n_keys, per_key = (40, 6) if batch_size == 1 else (900, 40)
    key, val, off = stream(11 + batch_size, n_keys, per_key, vmax, redeliver=0.03)
    ir = mk().to_ir(PL.I32)
    want = oracle_forwards(ir, key, val, off)
    t = drive(jl, ir, key, val, off, batch_size, max_keys=n_keys)
    assert t.path == expect_path
    assert len(want) > 0 and t.forwarded == want
    assert jl.pins() == 0


def test_unflagged_stencil_carry_batch_is_refused(jl):
    """Without CEP_BATCH_OFFSETS_MONOTONE a stencil carry session cannot apply the high-water mark
    to its halo and refuses the batch -- what every round-2 Java flush of C2/C5 hit."""
    ir = synth.c2_pattern().to_ir(PL.I32)
    p = jl.cepCompile(ir)
    s = jl.cepSessionOpen(p, 0, 1, 16, 1, 4, 0, 0)
    assert s > 0 and jl.cepSessionPath(s) == 1
    z = np.zeros(4, np.int32)
    args = (s, 4, np.array([0, 0, 1, 1], np.int32), z, z, np.arange(4, dtype=np.int64), np.arange(4, dtype=np.int64),
            np.array([1], np.int32), [np.array([0, 1, 2, 3], np.int32)])
    assert jl.cepPushBatch(*args, 0) == 12                    # CEP_E_UNSUPPORTED
    assert "MONOTONE" in jl.cepLastError()
    assert jl.cepPushBatch(*args, 1) == 0
    jl.cepSessionClose(s)
    jl.cepPatternFree(p)
    assert jl.pins() == 0


def test_capacity_keys_are_rerun_not_dropped(jl):
    """A skip-till-any key that outgrows max_key_words is handed back (CEP_E_RUN_CAPACITY) and the
    twin re-pushes its records with the cap lifted: every match is forwarded, as the reference's."""
    rng = np.random.default_rng(9)
    lens = np.full(30, 10)
    lens[4] = 260                                             # the exploding key
    key = np.repeat(np.arange(30, dtype=np.int32), lens)
    rng.shuffle(key)
    val = rng.integers(0, 4, len(key)).astype(np.int32)
    off = np.arange(len(key), dtype=np.int64)
    ir = PL.any_any().to_ir(PL.I32)
    want = oracle_forwards(ir, key, val, off)
    t = drive(jl, ir, key, val, off, 200, max_keys=30, max_key_words=1 << 15)
    assert t.reruns > 0
    assert t.forwarded == want


@pytest.mark.parametrize("mk,vmax", [(synth.c2_pattern, 4), (PL.c3_stock, 7), (PL.any_any, 4)],
                         ids=["stencil", "runs_general", "general"])
def test_more_keys_than_ids_spill_and_return(jl, mk, vmax):
    """600 keys through a session of 64 key ids: the least recently used keys are spilled to the
    host and come back under other ids with their runs, buffer and high-water marks intact."""
    key, val, off = stream(21, 600, 12, vmax, redeliver=0.02)
    if mk is PL.c3_stock:
        val = (100 + np.cumsum(np.random.default_rng(2).integers(-5, 6, len(key)))).astype(np.int32)
    ir = mk().to_ir(PL.I32)
    want = oracle_forwards(ir, key, val, off)
    t = drive(jl, ir, key, val, off, 50, max_keys=64, prune_at=400)
    assert len(t.spilled) > 0 or t.next_id == 64
    assert len(want) > 0 and t.forwarded == want
    assert jl.pins() == 0
