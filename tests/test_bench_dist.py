"""world_size-2 gloo rehearsal of bench.py's multi-GPU logic on CPU.

Each rank builds its key shard with bench.shard, matches it with the oracle
(standing in for the device kernel, which needs a GPU), and reduces with
bench.gather_stats.  The sharded totals must equal one node-wide run over the
union of the shards: keys are disjoint, so per-key NFAs never cross ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N, K = 40_000, 2_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_matches(rank):
    import bench
    import oracle as O
    from kcep import synth, Schema
    ko, lo = bench.shard(rank, N, K)
    key, val, order = synth.c2_stream_np(N, K, key_offset=ko, lo=lo)
    p = O.OraclePattern(synth.c2_pattern().to_ir(Schema([("value", "i32")])))
    nm, cs = O.baseline(p, O.BatchArrays(key, [val], [1], offset=order, ts=order), O.MODE_PROCESSOR, 1)
    return key, nm, cs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    key, nm, _ = _shard_matches(rank)
    stats = torch.tensor([float(len(key)), float(nm), 0.5 + rank], dtype=torch.float64)
    tot = bench.gather_stats(stats, world)
    q.put((rank, int(key.min()), int(key.max()), nm, tot))
    dist.destroy_process_group()


def test_two_rank_key_sharding_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (r0, lo0, hi0, m0, t0), (r1, lo1, hi1, m1, t1) = res
    assert hi0 < lo1                                    # disjoint key ranges
    assert t0 == t1 == (2.0 * N, float(m0 + m1), 1.5)   # every rank sees the same totals, max time
    # the same totals as one process over the union of both shards
    import oracle as O
    from kcep import synth, Schema
    import bench
    parts = [synth.c2_stream_np(N, K, key_offset=bench.shard(r, N, K)[0], lo=bench.shard(r, N, K)[1]) for r in (0, 1)]
    key, val, order = (np.concatenate([a[i] for a in parts]) for i in range(3))
    p = O.OraclePattern(synth.c2_pattern().to_ir(Schema([("value", "i32")])))
    nm, _ = O.baseline(p, O.BatchArrays(key, [val], [1], offset=order, ts=order), O.MODE_PROCESSOR, 2)
    assert nm == m0 + m1 and m0 > 0 and m1 > 0


def test_single_rank_gather_is_identity():
    import bench
    assert bench.gather_stats(torch.tensor([3.0, 2.0, 1.0], dtype=torch.float64), 1) == (3.0, 2.0, 1.0)
