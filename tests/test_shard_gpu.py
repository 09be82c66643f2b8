"""Key-hash sharding on the device: cep_partition / cep_gather kernels against the host
partitioner, one batch split into two shards matched by two sessions against one session over
the whole batch, and the per-batch RCCL count exchange (single-rank group on the test GPU)."""
import os
import socket

import numpy as np
import pytest
import torch

from kcep import Schema, synth
from kcep import native as N
from kcep import shard as S

pytestmark = pytest.mark.gpu
I32 = Schema([("value", "i32")])


def csr(out):
    return {k: np.asarray(out[k]) for k in ("match_record", "match_key", "ent_off", "ent_name", "ent_record")}


def same(a, b):
    return all(np.array_equal(a[k], b[k]) for k in a)


@pytest.mark.parametrize("G", [1, 2, 7, 8, 64])
def test_device_partition_matches_host(G):
    key, _, _ = synth.c2_stream_np(300_001, 20_000)
    dev = torch.from_numpy(key).cuda()
    hp, ho = S.partition(key, G)
    dp, do = S.partition(dev, G, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(dp.cpu().numpy(), hp) and np.array_equal(do.cpu().numpy(), ho)
    table = np.random.default_rng(G).integers(0, G, 20_000).astype(np.int32)
    hp, ho = S.partition(key, G, table)
    dp, do = S.partition(dev, G, torch.from_numpy(table).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dp.cpu().numpy(), hp) and np.array_equal(do.cpu().numpy(), ho)
    for dt in (torch.int32, torch.int64, torch.uint8):
        src = torch.arange(len(key), device="cuda").to(dt)
        got = S.take(src, dp)
        torch.cuda.synchronize()
        assert torch.equal(got, src[dp])


def test_empty_batch_partition():
    dp, do = S.partition(torch.zeros(0, dtype=torch.int32, device="cuda"), 4)
    torch.cuda.synchronize()
    assert dp.numel() == 0 and do.cpu().tolist() == [0] * 5


CASES = [("c2", synth.c2_pattern, lambda: synth.c2_stream_np(2_000_000, 50_000)[:2]),
         ("c5", synth.c5_pattern, lambda: synth.c5_stream_np(20_000, L=100)[:2]),
         ("c4", synth.c4_pattern, lambda: synth.c4_stream_np(5_000, L=12)[:2]),
         ("c3", synth.c3_pattern, lambda: synth.c3_stream_np(5_000, L=100)[:2])]


@pytest.mark.parametrize("name,pat,stream", CASES, ids=[c[0] for c in CASES])
def test_two_sessions_equal_one(name, pat, stream):
    """Split one device-resident batch into two shards (device partitioner), match each shard in
    its own session, renumber and merge: the CSR of one session over the whole batch."""
    key, val = stream()
    ir = pat().to_ir(I32)
    cp = N.CompiledPattern(ir)
    st = torch.cuda.current_stream().cuda_stream
    dk, dv = torch.from_numpy(key).cuda(), torch.from_numpy(val).cuda()
    whole = N.Session(cp, len(key))
    whole.push(len(key), dk.data_ptr(), [dv.data_ptr()], mem=N.MEM_DEVICE, stream=st)
    want = csr(whole.collect())
    assert len(want["match_record"]) > 0
    outs = []
    for r in range(2):
        sh = S.split(r, 2, dk, [dv], stream=st)
        s = N.Session(cp, max(1, sh.n))
        assert s.path == whole.path
        s.push(sh.n, sh.key.data_ptr(), [c.data_ptr() for c in sh.cols], mem=N.MEM_DEVICE, stream=st)
        outs.append(S.globalize(csr(s.collect()), sh.perm))
        assert np.all(S.key_shard(int(sh.key[0]), 2) == r)
    assert same(S.merge(outs), want)


def test_count_exchange_single_rank():
    """CountExchange's device-side slot copy, side-stream all-gather and scan (one-rank RCCL group)."""
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        key, val, _ = synth.c2_stream_np(1_000_000, 30_000)
        cp = N.CompiledPattern(synth.c2_pattern().to_ir(I32))
        sess = N.Session(cp, len(key))
        dk, dv = torch.from_numpy(key).cuda(), torch.from_numpy(val).cuda()
        stream = torch.cuda.current_stream()
        ex = S.CountExchange(torch.device("cuda", 0))
        slots = []
        for n in (len(key), len(key) // 2, 1000):
            sess.push(n, dk.data_ptr(), [dv.data_ptr()], mem=N.MEM_DEVICE, stream=stream.cuda_stream)
            slots.append((ex.post(sess, n, stream), n, sess.checksum()[0]))
        for slot, n, nm in slots:
            assert ex.result(slot) == (0, n, nm)
        counts, off, tev, tm = S.exchange_counts(1000, slots[-1][2])
        assert counts.tolist() == [[1000, slots[-1][2]]] and off == 0
    finally:
        dist.destroy_process_group()
