"""Key-hash sharding (kcep/shard.py, cep_partition / cep_shard_plan / cep_gather) on the host.

The reference's keys never share state (Kafka key partitioning, README.md:348-355; per-key
run counter NFAStates.java:36), so a batch split by key shard and matched shard by shard must
emit exactly the matches of one run over the whole batch, in the same order once merged.
The world_size-2 gloo test drives the product partitioner and exchange of kcep/shard.py; the
oracle stands in for the device per shard (these tests have no GPU)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from kcep import Schema, synth
from kcep import shard as S
import patterns_lib as PL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fmix32(k):
    h = np.asarray(k, np.int64).astype(np.uint32).astype(np.uint64)
    h ^= h >> np.uint64(16); h = (h * np.uint64(0x85ebca6b)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13); h = (h * np.uint64(0xc2b2ae35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def test_key_shard_is_fmix32_mod():
    keys = np.array([0, 1, 2, 12345, -7, 2**31 - 1], np.int32)
    for G in (1, 2, 3, 8):
        assert [S.key_shard(int(k), G) for k in keys] == list((fmix32(keys) % np.uint64(G)).astype(int))


@pytest.mark.parametrize("G", [1, 2, 5, 8])
def test_host_partition_is_a_stable_split(G):
    rng = np.random.default_rng(G)
    key = np.sort(rng.integers(0, 500, 20_000)).astype(np.int32)
    perm, off = S.partition(key, G)
    assert off[0] == 0 and off[-1] == len(key) and np.all(np.diff(off) >= 0)
    assert sorted(perm.tolist()) == list(range(len(key)))
    want = (fmix32(key) % np.uint64(G)).astype(np.int64)
    for s in range(G):
        p = perm[off[s]:off[s + 1]]
        assert np.all(want[p] == s) and np.all(np.diff(p) > 0)    # its keys only, batch order
    table = rng.integers(0, G, 500).astype(np.int32)
    perm, off = S.partition(key, G, table)
    for s in range(G):
        assert np.all(table[key[perm[off[s]:off[s + 1]]]] == s)


def test_shard_plan_rebalances_to_equal_events():
    rng = np.random.default_rng(1)
    ev = rng.zipf(1.6, 5000).astype(np.int64)                      # skewed keys
    ev[:3] = [5000, 4000, 3000]
    t0, l0 = S.shard_plan(ev, 8, rebalance=False)
    assert list(t0) == [S.key_shard(k, 8) for k in range(len(ev))]
    t1, l1 = S.shard_plan(ev, 8, rebalance=True)
    assert l0.sum() == l1.sum() == ev.sum()
    assert all(l1[s] == ev[t1 == s].sum() for s in range(8))
    assert l1.max() < l0.max() and l1.max() - l1.min() <= max(ev.max(), 1)
    assert t1.min() >= 0 and t1.max() < 8


def test_take_gathers_every_width():
    rng = np.random.default_rng(2)
    perm = rng.permutation(1000)[:300]
    for dt in (np.uint8, np.int32, np.int64, np.float64):
        a = rng.integers(0, 100, 1000).astype(dt)
        assert np.array_equal(S.take(a, perm), a[perm])


def oracle_csr(ir, key, cols, coltypes, mode=O.MODE_PROCESSOR, **kw):
    p = O.OraclePattern(ir)
    r = O.OracleRun(p, mode)
    r.process(O.BatchArrays(key, cols, coltypes, **kw))
    ms = r.matches(with_groups=False)
    ent = [t for m in ms for t in m.traversal]
    off = np.zeros(len(ms) + 1, np.int64)
    np.cumsum([len(m.traversal) for m in ms], out=off[1:])
    return dict(match_record=np.array([m.record for m in ms], np.int64),
                match_key=np.array([m.key for m in ms], np.int32), ent_off=off,
                ent_name=np.array([e[0] for e in ent], np.int32), ent_record=np.array([e[1] for e in ent], np.int64))


def same(a, b):
    return all(np.array_equal(a[k], b[k]) for k in ("match_record", "match_key", "ent_off", "ent_name", "ent_record"))


CASES = [("c2", lambda: synth.c2_pattern(), lambda: synth.c2_stream_np(60_000, 3_000)[:2]),
         ("c5", lambda: synth.c5_pattern(), lambda: synth.c5_stream_np(600, L=100)[:2]),
         ("c4", lambda: synth.c4_pattern(), lambda: synth.c4_stream_np(800, L=12)[:2]),
         ("c3", lambda: synth.c3_pattern(), lambda: synth.c3_stream_np(300, L=100)[:2])]


@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("name,pat,stream", CASES, ids=[c[0] for c in CASES])
def test_shards_merge_to_the_whole_batch(name, pat, stream, G):
    """Each shard matched on its own (oracle) and merged == one run over the batch."""
    key, val = stream()
    ir = pat().to_ir(Schema([("value", "i32")]))
    whole = oracle_csr(ir, key, [val], [1])
    assert len(whole["match_record"]) > 0
    outs = []
    for r in range(G):
        sh = S.split(r, G, key, [val])
        outs.append(S.globalize(oracle_csr(ir, sh.key, sh.cols, [1]), sh.perm))
    assert same(S.merge(outs), whole)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, val = synth.c5_stream_np(900, L=100)[:2]            # the node-wide batch every rank sees
        ir = synth.c5_pattern().to_ir(Schema([("value", "i32")]))
        table, _ = S.shard_plan(np.bincount(key, minlength=900), world, rebalance=True)
        sh = S.split(rank, world, key, [val], table=table)          # the product partitioner
        out = oracle_csr(ir, sh.key, sh.cols, [1])                  # stands in for this rank's GPU
        counts, off, tot_ev, tot_m = S.exchange_counts(sh.n, len(out["match_record"]))
        merged = S.gather_matches(out, sh.perm, dst=0)
        q.put((rank, sh.n, len(out["match_record"]), counts.tolist(), off, tot_ev, tot_m,
               None if merged is None else {k: v.tolist() for k, v in merged.items()}))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_matching_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (r0, n0, m0, c0, o0, e0, t0, merged), (r1, n1, m1, c1, o1, e1, t1, none) = res
    assert none is None and c0 == c1 == [[n0, m0], [n1, m1]]
    assert (o0, o1) == (0, m0) and e0 == e1 == n0 + n1 == 90_000 and t0 == t1 == m0 + m1
    assert n0 > 0 and n1 > 0 and abs(n0 - n1) <= 100                 # rebalanced to equal events
    key, val = synth.c5_stream_np(900, L=100)[:2]
    whole = oracle_csr(synth.c5_pattern().to_ir(Schema([("value", "i32")])), key, [val], [1])
    assert same({k: np.asarray(v) for k, v in merged.items()}, whole) and m0 > 0 and m1 > 0
