"""A key that outgrows the device continues on the reference NFA from its exported state.

The reference never runs out of capacity (NFA.java:134-149 over unbounded KV stores, NFAStoreImpl.java:
34-85).  The device hands a key that outgrows its workspace back per key (CEP_E_RUN_CAPACITY in
cep_batch_errors, its state kept as of the batch start); cep_state_evict gives that state as a KCST
blob and cep_state_to_reference rewrites it in the reference's own terms (NFA.runs, high-water marks,
the run queue with Dewey versions, buffer nodes with refs and ordered predecessors, aggregates --
NFAStates.java:33-109, MatchedEvent.java:27-169, AggregatesStoreImpl.java:30-76).  Here the oracle (the
C restatement of the reference NFA) imports that form and continues the key over the rest of its
records; the stream it then produces, joined to what the device emitted before the hand-off, must be
the uninterrupted reference run's, match for match.
"""
import struct

import numpy as np
import pytest

import oracle as O
from kcep import Schema, QueryBuilder, Selected, Event, States, Curr
from kcep import native as N
from kcep import synth
import patterns_lib as PL

pytestmark = pytest.mark.gpu

RUN_CAPACITY = 9


def parse_kcrf_events(blob):
    """The events of a KCRF blob: [(position, topic, partition, offset, ts, [col bits])]."""
    magic, ver, key, ncols, runs = struct.unpack_from("<IIiiq", blob, 0)
    assert magic == 0x4652434B and ver == 1
    at = 24
    (nh,) = struct.unpack_from("<i", blob, at)
    at += 4 + 12 * nh
    (ne,) = struct.unpack_from("<i", blob, at)
    at += 4
    evs = []
    for _ in range(ne):
        pos, tp, part, off, ts = struct.unpack_from("<qiiqq", blob, at)
        at += 32
        cols = list(struct.unpack_from("<%dq" % ncols, blob, at))
        at += 8 * ncols
        evs.append((pos, tp, part, off, ts, cols))
    return key, runs, evs


def heavy_stream(seed, n_light=6):
    """Key 0 explodes on skip-till-any (C4 shape); keys 1..n_light stay light.  Arrival order,
    offset = arrival index per (single) topic partition."""
    rng = np.random.default_rng(seed)
    recs = []
    heavy = [0] + list(rng.choice([1, 1, 2, 2, 3, 0], 30))
    light = {k: list(rng.integers(0, 4, 12)) for k in range(1, n_light + 1)}
    order = [0] * len(heavy) + [k for k in light for _ in light[k]]
    rng.shuffle(order[1:])
    it = {0: iter(heavy), **{k: iter(v) for k, v in light.items()}}
    for k in order:
        recs.append((k, int(next(it[k]))))
    return [(k, v, i) for i, (k, v) in enumerate(recs)]     # (key, value, offset)


def oracle_all(ir, recs):
    r = O.OracleRun(O.OraclePattern(ir), O.MODE_PROCESSOR)
    key = np.array([x[0] for x in recs], np.int32)
    val = np.array([x[1] for x in recs], np.int32)
    off = np.array([x[2] for x in recs], np.int64)
    r.process(O.BatchArrays(key, [val], [1], offset=off, ts=off))
    out = {}
    for m in r.matches(with_groups=False):
        out.setdefault(int(key[m.record]), []).append((int(off[m.record]), [(nm, int(off[e])) for nm, e in m.traversal]))
    return out


def run_with_handoff(ir, recs, nbatch, cap_words):
    """Push `recs` (arrival order) in `nbatch` batches through a carry session whose per-key workspace is
    capped; a key handed back with CEP_E_RUN_CAPACITY continues on the oracle from its exported state.
    Returns (matches per key as (completing offset, [(name, offset)]), hand-off batch, blob)."""
    pat = N.CompiledPattern(ir)
    s = N.Session(pat, len(recs), mode=N.MODE_PROCESSOR, carry=True, max_keys=16, max_key_words=cap_words)
    assert s.path == N.PATH_GENERAL
    bounds = np.linspace(0, len(recs), nbatch + 1).astype(int)
    got, pos_off = {}, {}
    cpu_key, handoff, ref_blob = None, None, None
    for bi, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        batch = [x for x in recs[a:b] if x[0] != cpu_key]
        batch.sort(key=lambda x: x[0])                     # grouped by key, arrival order per key (stable)
        base = s.stream_position()
        for j, x in enumerate(batch):
            pos_off[base + j] = x[2]
        key = np.array([x[0] for x in batch], np.int32)
        val = np.array([x[1] for x in batch], np.int32)
        off = np.array([x[2] for x in batch], np.int64)
        s.push(len(batch), key, [val], offset=off, ts=off, flags=N.BATCH_OFFSETS_MONOTONE)
        out = s.collect(raise_on_error=False)
        erec, ecode = s.batch_errors()
        cap_keys = {int(key[r - base]) for r, c in zip(erec, ecode) if c == RUN_CAPACITY}
        assert all(c == RUN_CAPACITY for c in ecode)
        for m in range(len(out["match_record"])):
            k = int(out["match_key"][m])
            if k in cap_keys:
                continue
            e0, e1 = out["ent_off"][m], out["ent_off"][m + 1]
            ents = [(int(out["ent_name"][i]), pos_off[int(out["ent_record"][i])]) for i in range(e0, e1)]
            got.setdefault(k, []).append((pos_off[int(out["match_record"][m])], ents))
        if cap_keys and (cpu_key is not None or cap_keys != {0}):
            return None, None, None                          # the cap is too small for the light keys too
        if cap_keys:
            cpu_key, handoff = 0, bi
            ref_blob = s.state_evict([0])[0]                 # its state as of this batch's start
            rest = [x for x in recs[a:] if x[0] == 0]        # its records from this batch on
            if ref_blob:
                ref = pat.state_to_reference(ref_blob)
                _, _, evs = parse_kcrf_events(ref)
            else:                                            # handed back in its first batch: no state yet
                ref, evs = None, []
            key = np.array([0] * (len(evs) + len(rest)), np.int32)
            val = np.array([e[5][0] for e in evs] + [x[1] for x in rest], np.int32)
            off = np.array([e[3] for e in evs] + [x[2] for x in rest], np.int64)
            ts = np.array([e[4] for e in evs] + [x[2] for x in rest], np.int64)
            r = O.OracleRun(O.OraclePattern(ir), O.MODE_PROCESSOR)
            bat = O.BatchArrays(key, [val], [1], offset=off, ts=ts)
            if ref is not None:
                r.resume(bat, ref)
            else:
                r.process(bat)
            for m in r.matches(with_groups=False):
                got.setdefault(0, []).append((int(off[m.record]), [(nm, int(off[e])) for nm, e in m.traversal]))
            ref_blob = ref
    return got, handoff, ref_blob


@pytest.mark.parametrize("seed", [1, 2])
def test_capacity_key_continues_on_the_reference(seed):
    """C4's skip-till-any shape: the heavy key exhausts a deliberately small per-key workspace mid-stream
    and is continued by the oracle from cep_state_to_reference; the result equals an uninterrupted run."""
    ir = synth.c4_pattern().to_ir(Schema([("value", "i32")]))
    recs = heavy_stream(seed)
    want = oracle_all(ir, recs)
    assert len(want.get(0, [])) > 10
    tried = []
    for cap in np.unique(np.geomspace(300, 300_000, 40).astype(int)):
        got, handoff, ref = run_with_handoff(ir, recs, 6, int(cap))
        tried.append((int(cap), None if got is None else handoff))
        if got is not None and handoff is not None and handoff >= 1 and ref:
            break
    else:
        pytest.fail(f"no per-key cap made the heavy key hand off after its first batch: {tried}")
    for k in set(want) | set(got):
        assert sorted(got.get(k, [])) == sorted(want.get(k, [])), k
    # per-key emission order: the device's matches, then the reference's, each in the reference's order
    assert [m for m in got[0]] == want[0]
    key, runs, evs = parse_kcrf_events(ref)
    assert key == 0 and runs >= 1 and len(evs) > 0


def test_stateful_key_continues_on_the_reference():
    """The stock demo (folds, States.get/getOrElse, skip-till-next oneOrMore): aggregates and their
    sequences cross the hand-off too."""
    sch = PL.STOCK_SCHEMA
    ir = PL.stock_demo().to_ir(sch)
    rng = np.random.default_rng(7)
    n = 60
    price = (100 + np.cumsum(rng.integers(-3, 4, n))).astype(np.int64)
    vol = rng.integers(900, 1400, n).astype(np.int64)
    pat = N.CompiledPattern(ir)
    # one key; after batch 1, evict and continue on the oracle
    s = N.Session(pat, n, mode=N.MODE_PROCESSOR, carry=True, max_keys=4)
    k = np.zeros(n, np.int32)
    off = np.arange(n, dtype=np.int64)
    cut = 25
    s.push(cut, k[:cut], [price[:cut], vol[:cut]], offset=off[:cut], ts=off[:cut], flags=N.BATCH_OFFSETS_MONOTONE)
    out = s.collect(raise_on_error=False)
    assert out["err"] == 0
    first = [(int(out["match_record"][m]),
              [(int(out["ent_name"][i]), int(out["ent_record"][i])) for i in range(out["ent_off"][m], out["ent_off"][m + 1])])
             for m in range(len(out["match_record"]))]
    blob = s.state_evict([0])[0]
    ref = pat.state_to_reference(blob)
    _, _, evs = parse_kcrf_events(ref)
    r = O.OracleRun(O.OraclePattern(ir), O.MODE_PROCESSOR)
    E = len(evs)
    key = np.zeros(E + n - cut, np.int32)
    cols = [np.array([struct.unpack("<q", struct.pack("<q", e[5][c]))[0] for e in evs] + list(col[cut:]), np.int64)
            for c, col in enumerate((price, vol))]
    o2 = np.array([e[3] for e in evs] + list(off[cut:]), np.int64)
    r.resume(O.BatchArrays(key, cols, [2, 2], offset=o2, ts=o2), ref)
    second = [(int(o2[m.record]), [(nm, int(o2[e])) for nm, e in m.traversal]) for m in r.matches(with_groups=False)]
    w = O.OracleRun(O.OraclePattern(ir), O.MODE_PROCESSOR)
    w.process(O.BatchArrays(k, [price, vol], [2, 2], offset=off, ts=off))
    want = [(m.record, [(nm, e) for nm, e in m.traversal]) for m in w.matches(with_groups=False)]
    assert first + second == want and len(second) > 0
