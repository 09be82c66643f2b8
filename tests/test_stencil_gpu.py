"""Parity of the HIP stencil path (csrc/stencil.hip) with the CPU oracle.

Every test calls libkcep.so through the C-ABI on cuda:0 and compares the
emitted matches (emitting record, key, and the full shared-buffer traversal:
stage name + record, final stage first) bit-exactly with oracle/cep_oracle.c
on the same seeded inputs."""
import numpy as np
import pytest

import oracle as O
from kcep import native as N
from kcep import synth, Schema, QueryBuilder, Event, Selected
from golden_util import scenarios, event_arrays
from gpu_util import oracle_matches, run_product

pytestmark = pytest.mark.gpu

I32 = Schema([("value", "i32")])


def c2_ir():
    return synth.c2_pattern().to_ir(I32)


@pytest.mark.parametrize("name", ["nfa_strict3", "readme_letters"])
def test_golden_stencil(name):
    fx = [f for f in scenarios() if f["name"] == name][0]
    a = event_arrays(fx)
    ir = bytes.fromhex(fx["ir"])
    key = a["key"] if fx["mode"] == O.MODE_PROCESSOR else np.zeros_like(a["key"])   # single NFA = one key
    want = oracle_matches(ir, key, a["cols"], a["coltypes"], fx["mode"], topic=a["topic"],
                          partition=a["partition"], offset=a["offset"], ts=a["ts"])
    got, s = run_product(ir, key, a["cols"], mode=fx["mode"], topic=a["topic"], flags=N.BATCH_OFFSETS_MONOTONE)
    assert s.path == N.PATH_STENCIL
    assert got == want
    assert len(got) == len(fx["expected"]["sequences"])


@pytest.mark.parametrize("kernel", ["plain", "keyed"])
@pytest.mark.parametrize("n,K", [(0, 1), (1, 1), (2, 1), (3, 1), (4095, 3), (4096, 7), (4097, 1), (8191, 50),
                                 (12289, 13), (100_003, 1000), (200_000, 100_000), (65_537, 1)])
def test_c2_random(n, K, kernel, monkeypatch):
    """Both stencil kernels on resident batches: the keyless plain one (the default for k <= 7) and the
    keyed one carry sessions run (KCEP_STENCIL_KEYED=1 routes a resident batch through it)."""
    monkeypatch.setenv("KCEP_STENCIL_KEYED", "1" if kernel == "keyed" else "0")
    key, val, order = synth.c2_stream_np(n, K)
    ir = c2_ir()
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR, offset=order, ts=order)
    got, _ = run_product(ir, key, [val])
    assert got == want


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
def test_k_stages(k):
    rng = np.random.default_rng(k)
    n = 50_000
    key = np.sort(rng.integers(0, 300, n)).astype(np.int32)
    val = rng.integers(0, 3, n).astype(np.int32)          # dense hits: long overlapping runs
    q = QueryBuilder().select("s0").where(Event.value() <= (0 if k > 1 else 1))
    for s in range(1, k):
        q = q.then().select(f"s{s}").where((Event.value() == s % 3) | (Event.value() == 2))
    ir = q.build().to_ir(I32)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    got, s = run_product(ir, key, [val])
    assert s.path == N.PATH_STENCIL
    assert got == want and len(got) > 0


def test_always_true_overlapping_matches():
    n = 20_000
    key = (np.arange(n) // 37).astype(np.int32)
    val = np.zeros(n, np.int32)
    ir = (QueryBuilder().select("a").where(True).then().select("b").where(True).then()
          .select("c").where(True).build().to_ir(I32))
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR)
    got, _ = run_product(ir, key, [val])
    assert got == want and len(got) == n - 2 * len(np.unique(key))


def test_match_dense_super_tiles():
    """The plain kernel's slot layout at four tiles per workgroup (>= 8192 tiles): a super-tile's first
    ST_DENSE (512) matches in the dense region, the rest in its own region, a tile whose matches no
    longer fit the LDS staging (over 4096) stored straight to both (csrc/stencil_kernel.h STAGE).
    Per super-tile: tile 0 no match (distinct keys), tile 1 400 matches, tiles 2-3 ~3.8 k each."""
    import os
    import torch
    n = 8192 * 4096 + 1000
    r = np.arange(n) % 16384
    t, o = r // 4096, r % 4096
    new = (t == 0) | ((t == 1) & ((o == 0) | (o >= 402))) | ((t >= 2) & (o % 37 == 0))
    key = (np.cumsum(new) - 1).astype(np.int32)
    val = np.zeros(n, np.int32)
    ir = (QueryBuilder().select("a").where(True).then().select("b").where(True).then()
          .select("c").where(True).build().to_ir(I32))
    s = N.Session(N.CompiledPattern(ir), n)
    assert s.path == N.PATH_STENCIL
    dk, dv = torch.from_numpy(key).cuda(), torch.from_numpy(val).cuda()
    s.push(n, dk.data_ptr(), [dv.data_ptr()], mem=N.MEM_DEVICE, stream=torch.cuda.current_stream().cuda_stream)
    got = s.collect()
    b = O.BatchArrays(key, [val], [1])
    want = O.baseline_csr(O.OraclePattern(ir), b, O.MODE_PROCESSOR, min(16, os.cpu_count() or 1))
    assert len(want["match_record"]) > 10_000_000
    for f in ("match_record", "match_key", "ent_off", "ent_name", "ent_record"):
        assert got[f].shape == want[f].shape, f
        bad = np.flatnonzero(got[f] != want[f])
        assert len(bad) == 0, (f, bad[:5], got[f][bad[:5]], want[f][bad[:5]])


@pytest.mark.parametrize("t", ["i64", "f64"])
def test_wide_columns(t):
    rng = np.random.default_rng(7)
    n = 60_000
    key = np.sort(rng.integers(0, 500, n)).astype(np.int32)
    raw = rng.integers(-5, 6, n)
    val = (raw * 1_000_000_007).astype(np.int64) if t == "i64" else raw.astype(np.float64) * 0.5
    sch = Schema([("value", t)])
    c = 1_000_000_007 if t == "i64" else 0.5
    q = (QueryBuilder().select("lo").where(Event.value() < 0).then()
         .select("mid").where((Event.value() >= 0) & (Event.value() <= c * 2)).then()
         .select("hi").where(Event.value() > c).build())
    ir = q.to_ir(sch)
    ty = 2 if t == "i64" else 3
    want = oracle_matches(ir, key, [val], [ty], O.MODE_PROCESSOR)
    got, s = run_product(ir, key, [val])
    assert s.path == N.PATH_STENCIL
    assert got == want and len(got) > 0


def test_topic_filter():
    rng = np.random.default_rng(3)
    n = 40_000
    key = np.sort(rng.integers(0, 400, n)).astype(np.int32)
    val = rng.integers(0, 3, n).astype(np.int32)
    topic = rng.integers(0, 2, n).astype(np.int32)
    sch = Schema([("value", "i32")], topics=["t0", "t1"])
    q = (QueryBuilder().select("a", Selected.withStrictContiguity().withTopic("t1")).where(Event.value() == 0)
         .then().select("b").where(Event.value() != 0).then()
         .select("c", Selected.withStrictContiguity().withTopic("t0")).where(Event.value() == 2).build())
    ir = q.to_ir(sch)
    want = oracle_matches(ir, key, [val], [1], O.MODE_PROCESSOR, topic=topic)
    got, s = run_product(ir, key, [val], topic=topic)
    assert s.path == N.PATH_STENCIL
    assert got == want and len(got) > 0


def test_device_resident_batch_and_checksum():
    import torch
    n, K = 5_000_000, 50_000
    key, val, order = synth.c2_stream_torch(n, K, "cuda")
    cp = N.CompiledPattern(c2_ir())
    s = N.Session(cp, n)
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE,
           stream=torch.cuda.current_stream().cuda_stream)
    nm, cs = s.checksum()
    hk, hv, ho = key.cpu().numpy(), val.cpu().numpy(), order.cpu().numpy()
    p = O.OraclePattern(c2_ir())
    b = O.BatchArrays(hk, [hv], [1], offset=ho, ts=ho)
    want_n, want_cs = O.baseline(p, b, O.MODE_PROCESSOR, 16)
    assert (nm, cs) == (want_n, want_cs)


def test_many_super_tiles_multi_workgroup_scan():
    """Over 8192 super-tiles (140 M records) the tile counts are scanned by the multi-workgroup
    exclusive_scan instead of tile_scan (csrc/stencil.hip stencil_launch)."""
    import torch
    n, K = 140_000_000, 1_000_000
    key, val, order = synth.c2_stream_torch(n, K, "cuda")
    cp = N.CompiledPattern(c2_ir())
    s = N.Session(cp, n)
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE,
           stream=torch.cuda.current_stream().cuda_stream)
    nm, cs = s.checksum()
    hk, hv, ho = key.cpu().numpy(), val.cpu().numpy(), order.cpu().numpy()
    del key, val, order, s
    b = O.BatchArrays(hk, [hv], [1], offset=ho, ts=ho)
    want_n, want_cs = O.baseline(O.OraclePattern(c2_ir()), b, O.MODE_PROCESSOR, 16)
    assert (nm, cs) == (want_n, want_cs) and nm > 1_000_000


def test_irregular_batches_route_to_general_path():
    """Null records and unflagged offsets break the stencil's contiguity assumption:
    the session hands those batches to the general NFA kernel, with the same result."""
    from test_general_gpu import run_both
    import oracle as O
    rng = np.random.default_rng(3)
    key = np.repeat(np.arange(50, dtype=np.int32), 40)
    val = rng.integers(0, 3, len(key)).astype(np.int32)
    valid = (rng.random(len(key)) > 0.05).astype(np.uint8)
    off = np.arange(len(key), dtype=np.int64)
    for kw in (dict(valid=valid), dict(offset=off)):
        cp = N.CompiledPattern(c2_ir())
        s = N.Session(cp, len(key))
        assert s.path == N.PATH_STENCIL
        s.push(len(key), key, [val], **kw)
        out = s.collect()
        assert out["path"] == N.PATH_GENERAL
        want, got, oerr, gerr = run_both(c2_ir(), O.MODE_PROCESSOR, key, [val], [1], force=0, **kw)
        assert oerr is None and gerr is None and got == want and len(got) > 0
