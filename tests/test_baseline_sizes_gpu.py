"""Parity at BASELINE.json's full sizes: every config's device-resident batch through
the C-ABI against the oracle's multi-threaded run of the same records, by match count and the
checksum of every traversal (emitting record, stage names and records; cep_checksum / orc_baseline
hash them identically).  C2: 1 M keys x 100 M events; C3: 100 k stock keys x 100; C4: 100 k keys x
12 (skip-till-any run explosion); C5: 1.25 M keys x 100 (one GPU's share of the node-wide 10 M)."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from kcep import native as N, synth, Schema

pytestmark = pytest.mark.gpu

I32 = Schema([("value", "i32")])
THREADS = 16          # the GPU box's CPU share (cgroup quota); the oracle is key-sharded


def _cfg(name):
    dev = torch.device("cuda", 0)
    if name == "c2":
        key, val, order = synth.c2_stream_torch(100_000_000, 1_000_000, dev)
        return key, val, order, synth.c2_pattern(), N.PATH_STENCIL
    gen = {"c3": (synth.c3_stream_torch, 100_000, 100, synth.c3_pattern, N.PATH_RUNS),
           "c4": (synth.c4_stream_torch, 100_000, 12, synth.c4_pattern, N.PATH_GENERAL),
           "c5": (synth.c5_stream_torch, 1_250_000, 100, synth.c5_pattern, N.PATH_CHAIN)}[name]
    key, val, ts = gen[0](gen[1], dev, L=gen[2])
    return key, val, ts, gen[3](), gen[4]


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_full_size_checksum(name):
    key, val, ts, pat, path = _cfg(name)
    n = key.numel()
    ir = pat.to_ir(I32)
    s = N.Session(N.CompiledPattern(ir), n, mode=N.MODE_PROCESSOR)
    assert s.path == path
    st = torch.cuda.current_stream()
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=st.cuda_stream,
           ts=ts.data_ptr() if name != "c2" else None)
    gm, gcs = s.checksum()
    hk, hv, ht = key.cpu().numpy(), val.cpu().numpy(), ts.cpu().numpy()
    b = O.BatchArrays(hk, [hv], [1], offset=ht if name == "c2" else None, ts=ht)
    om, ocs = O.baseline(O.OraclePattern(ir), b, O.MODE_PROCESSOR, min(THREADS, os.cpu_count() or 1))
    assert gm == om and gcs == ocs and gm > 0


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_full_size_ordered_csr(name):
    """Element by element, not only the order-independent checksum: every match's emitting record, key
    and traversal (stage name, record), in the CSR's order -- key order of the grouped batch, per key
    the reference's emission order (CEPProcessor.java:148, SharedVersionedBufferStoreImpl.peek) -- at
    the full sizes of every config, against the oracle's run of the same records.  C3 exercises the runs
    path's ordering (runs_order's windowed rank in LDS, runs.hip), C4 the wave kernel's queue-order
    placement by prefix scans (nfa_wave.h) and its matchConstruction walks."""
    key, val, ts, pat, path = _cfg(name)
    n = key.numel()
    ir = pat.to_ir(I32)
    s = N.Session(N.CompiledPattern(ir), n, mode=N.MODE_PROCESSOR)
    assert s.path == path
    st = torch.cuda.current_stream()
    s.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=st.cuda_stream,
           ts=ts.data_ptr() if name != "c2" else None)
    got = s.collect()
    hk, hv, ht = key.cpu().numpy(), val.cpu().numpy(), ts.cpu().numpy()
    del key, val, ts
    b = O.BatchArrays(hk, [hv], [1], offset=ht if name == "c2" else None, ts=ht)
    want = O.baseline_csr(O.OraclePattern(ir), b, O.MODE_PROCESSOR, min(THREADS, os.cpu_count() or 1))
    assert len(want["match_record"]) > {"c2": 1_000_000, "c3": 1_000_000, "c4": 100_000, "c5": 1_000_000}[name]
    for f in ("match_record", "match_key", "ent_off", "ent_name", "ent_record"):
        assert got[f].shape == want[f].shape, f
        bad = np.flatnonzero(got[f] != want[f])
        assert len(bad) == 0, (f, bad[:5], got[f][bad[:5]], want[f][bad[:5]])
