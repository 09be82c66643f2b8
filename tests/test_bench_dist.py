"""world_size-2 gloo rehearsal of bench.py's multi-GPU logic on CPU.

Each rank builds the node-wide stream and takes its shard with bench.workload -- the product
partitioner (cep_shard_plan + cep_partition / cep_gather through kcep/shard.py), here on CPU
tensors -- matches it with the oracle (standing in for the device kernel, which needs a GPU)
and reduces with bench.gather_stats.  The sharded totals must equal one node-wide run:
per-key NFAs never cross ranks."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N, K = 40_000, 2_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    for p in (ROOT, os.path.join(ROOT, "kafkastreams-cep_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import oracle as O
    key, cols, ts, ir, (sh, info) = bench.workload("c2", rank, world, K, N, torch.device("cpu"), None)
    p = O.OraclePattern(ir)
    nm, cs = O.baseline(p, O.BatchArrays(key.numpy(), [cols[0].numpy()], [1], offset=ts.numpy(), ts=ts.numpy()),
                        O.MODE_PROCESSOR, 1)
    stats = torch.tensor([float(len(key)), float(nm), 0.5 + rank], dtype=torch.float64)
    tot = bench.gather_stats(stats, world)
    q.put((rank, set(np.unique(key.numpy()).tolist()), len(key), nm, tot, info["planned_events"]))
    dist.destroy_process_group()


def test_two_rank_key_sharding_gloo():
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
    (r0, k0, n0, m0, t0, pl0), (r1, k1, n1, m1, t1, pl1) = res
    assert not (k0 & k1) and len(k0 | k1) == 2 * K       # every key on exactly one rank
    assert pl0 == pl1 == [n0, n1] and n0 + n1 == 2 * N   # the plan every rank computed, realised
    assert abs(n0 - n1) <= 100                           # equal-event rebalance
    assert t0 == t1 == (2.0 * N, float(m0 + m1), 1.5)    # every rank sees the same totals, max time
    # the same totals as one process over the node-wide stream
    import oracle as O
    from kcep import synth, Schema
    key, val, order = synth.c2_stream_np(2 * N, 2 * K)
    p = O.OraclePattern(synth.c2_pattern().to_ir(Schema([("value", "i32")])))
    nm, _ = O.baseline(p, O.BatchArrays(key, [val], [1], offset=order, ts=order), O.MODE_PROCESSOR, 2)
    assert nm == m0 + m1 and m0 > 0 and m1 > 0


def test_single_rank_gather_is_identity():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.gather_stats(torch.tensor([3.0, 2.0, 1.0], dtype=torch.float64), 1) == (3.0, 2.0, 1.0)
